"""Utterance sharding across ranks: one process per GPU, weights replicated, each
rank runs whole ``VC.pipeline`` calls on its share of the utterances; the only collective is the
gather of the variable-length output waveforms to rank 0 (RCCL over xGMI with backend "nccl",
gloo on CPU for the tests).

The reference processes a batch of files one ``pipeline()`` call at a time
(``convert.py:129-135``); calls share no state, so the split needs no data-path exchange.
"""
from __future__ import annotations

import heapq

import torch


def shard_utterances(lengths, world: int):
    """Greedy longest-first assignment to the least-loaded rank -> list of index lists per rank.

    Deterministic: ties in length keep input order, ties in load go to the lower rank."""
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))
    heap = [(0, r) for r in range(world)]
    shards = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        shards[r].append(i)
        heapq.heappush(heap, (load + int(lengths[i]), r))
    for s in shards:
        s.sort()
    return shards


def gather_waveforms(outs, dist, dst: int = 0, stats: dict | None = None):
    """Gather each rank's list of 1-D f32 waveforms to ``dst``: an all_gather of the int64
    counts and lengths, then one grouped send / recv per rank of exactly its waveforms' samples
    (``dist.batch_isend_irecv``: grouped ncclSend / ncclRecv over xGMI with backend "nccl", host sends with
    gloo) -- no padding travels, and dst's own waveforms do not move.  Returns the list of lists (per
    source rank) on ``dst`` and None elsewhere; ``stats`` (a dict) receives "bytes_sent" / "bytes_recv" of
    this rank's point-to-point traffic.  Works for any backend whose tensors live on ``outs``' device (nccl:
    cuda, gloo: cpu)."""
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = outs[0].device if outs else torch.device("cuda" if dist.get_backend() == "nccl" else "cpu")
    counts = torch.tensor([len(outs)], dtype=torch.int64, device=dev)
    all_counts = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(all_counts, counts)
    maxn = max(1, max(int(c) for c in all_counts))
    sizes = torch.zeros(maxn, dtype=torch.int64, device=dev)
    if outs:
        sizes[: len(outs)] = torch.tensor([o.numel() for o in outs], dtype=torch.int64)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes)
    lens = [[int(v) for v in all_sizes[r][: int(all_counts[r])]] for r in range(world)]
    total = [sum(ln) for ln in lens]
    p2p, bufs = [], {}
    if rank == dst:
        for r in range(world):
            if r != dst and total[r]:
                bufs[r] = torch.empty(total[r], dtype=torch.float32, device=dev)
                p2p.append(dist.P2POp(dist.irecv, bufs[r], r))
    elif total[rank]:
        flat = torch.cat([o.reshape(-1).float() for o in outs])
        p2p.append(dist.P2POp(dist.isend, flat, dst))
    if p2p:
        for req in dist.batch_isend_irecv(p2p):
            req.wait()
    if stats is not None:
        stats["bytes_sent"] = 4 * total[rank] if rank != dst else 0
        stats["bytes_recv"] = 4 * sum(total[r] for r in bufs) if rank == dst else 0
    if rank != dst:
        return None
    result = []
    for r in range(world):
        if r == dst:
            result.append([o.reshape(-1).float() for o in outs])
            continue
        parts, off = [], 0
        for ln in lens[r]:
            parts.append(bufs[r][off: off + ln] if ln else torch.empty(0, dtype=torch.float32, device=dev))
            off += ln
        result.append(parts)
    return result
