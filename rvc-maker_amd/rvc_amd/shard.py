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
    this rank's point-to-point traffic.  The waveforms stay on their device: with "nccl" the transport is that
    device; with gloo (CPU transport) device waveforms are packed on the device, staged through host memory
    and the received ones handed back on dst's device -- so a gloo run on GPU tensors executes every step of
    the "nccl" path except the transport itself."""
    rank, world = dist.get_rank(), dist.get_world_size()
    nccl = dist.get_backend() == "nccl"
    if outs:
        dev = outs[0].device
    else:
        dev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
    tdev = dev if nccl else torch.device("cpu")  # transport device
    counts = torch.tensor([len(outs)], dtype=torch.int64, device=tdev)
    all_counts = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(all_counts, counts)
    maxn = max(1, max(int(c) for c in all_counts))
    sizes = torch.zeros(maxn, dtype=torch.int64, device=tdev)
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
                bufs[r] = torch.empty(total[r], dtype=torch.float32, device=tdev)
                p2p.append(dist.P2POp(dist.irecv, bufs[r], r))
    elif total[rank]:
        flat = torch.cat([o.reshape(-1).float() for o in outs])  # packed on the waveforms' device
        p2p.append(dist.P2POp(dist.isend, flat.to(tdev), dst))
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
        buf = bufs[r].to(dev) if r in bufs else None
        parts, off = [], 0
        for ln in lens[r]:
            parts.append(buf[off: off + ln] if ln else torch.empty(0, dtype=torch.float32, device=dev))
            off += ln
        result.append(parts)
    return result


def convert_utterances(vc, model, net_g, sid, clips, shards, dist=None, pitch=0, version="v2", protect=0.33,
                       index=None, index_rate=0.0, f0_method="rmvpe", seed=17, stats=None, dst=0):
    """One rank's part of a sharded job (BASELINE configs[3]; the reference's file loop, convert.py:129-135):
    ``shards`` = ``shard_utterances(...)`` (utterance ids per rank), ``clips`` this rank's device inputs in the
    order of ``shards[rank]``.  The share runs as one clip stream in which utterance i draws its noise with seed
    ``seed + i`` -- keyed to the utterance, not to the rank or the stream position, so every utterance's waveform
    is the same bits whatever the world size -- then the waveforms are gathered to ``dst``.  Returns, on ``dst``,
    every utterance's waveform in utterance order (None elsewhere); without ``dist``, this rank's own."""
    rank = dist.get_rank() if dist is not None else 0
    mine = shards[rank]
    if len(clips) != len(mine):
        raise ValueError("convert_utterances: one clip per utterance of this rank's shard")
    outs = vc.pipeline_device_stream(model, net_g, sid, clips, pitch, version, protect, index, index_rate, f0_method,
                                     seeds=[seed + i for i in mine]) if clips else []
    if dist is None:
        return outs
    got = gather_waveforms(outs, dist, dst=dst, stats=stats)
    if got is None:
        return None
    n = sum(len(s) for s in shards)
    ordered = [None] * n
    for r, parts in enumerate(got):
        if len(parts) != len(shards[r]):
            raise RuntimeError(f"gather: rank {r} sent {len(parts)} waveforms for {len(shards[r])} utterances")
        for i, w in zip(shards[r], parts):
            ordered[i] = w
    return ordered
