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


def gather_waveforms(outs, dist, dst: int = 0):
    """Gather each rank's list of 1-D f32 waveforms to ``dst``.

    Lengths travel first (all_gather of int64 counts and sizes), then one padded buffer per rank
    (``dist.gather``).  Returns the list of lists (per source rank) on ``dst`` and None elsewhere.
    Works for any backend whose tensors live on ``outs``' device (nccl: cuda, gloo: cpu)."""
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = outs[0].device if outs else torch.device("cpu")
    n = len(outs)
    counts = torch.tensor([n], dtype=torch.int64, device=dev)
    all_counts = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(all_counts, counts)
    maxn = int(max(int(c) for c in all_counts))
    sizes = torch.zeros(maxn, dtype=torch.int64, device=dev)
    for i, o in enumerate(outs):
        sizes[i] = o.numel()
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes)
    total = [int(s.sum()) for s in all_sizes]
    cap = max(max(total), 1)
    buf = torch.zeros(cap, dtype=torch.float32, device=dev)
    if outs:
        flat = torch.cat([o.reshape(-1).float() for o in outs])
        buf[: flat.numel()] = flat
    bufs = [torch.zeros(cap, dtype=torch.float32, device=dev) for _ in range(world)] if rank == dst else None
    dist.gather(buf, bufs, dst=dst)
    if rank != dst:
        return None
    result = []
    for r in range(world):
        k = int(all_counts[r])
        lens = [int(v) for v in all_sizes[r][:k]]
        parts, off = [], 0
        for ln in lens:
            parts.append(bufs[r][off: off + ln])
            off += ln
        result.append(parts)
    return result
