"""Multi-rank utterance sharding + waveform gather, world_size 2 over gloo on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rvc_amd.shard import gather_waveforms, shard_utterances


def test_shard_longest_first_balances():
    lengths = [30, 10, 25, 5, 20, 15]
    shards = shard_utterances(lengths, 2)
    assert sorted(sum(shards, [])) == list(range(6))
    loads = [sum(lengths[i] for i in s) for s in shards]
    assert abs(loads[0] - loads[1]) <= 5
    assert shard_utterances(lengths, 2) == shards  # deterministic
    assert shard_utterances([7], 4) == [[0], [], [], []]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, lengths, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = shard_utterances(lengths, world)[rank]
        # each "utterance" output is a deterministic ramp identifying it
        outs = [torch.arange(lengths[i], dtype=torch.float32) + 1000 * i for i in mine]
        st = {}
        got = gather_waveforms(outs, dist, dst=0, stats=st)
        sent = torch.tensor([st["bytes_sent"], st["bytes_recv"]], dtype=torch.int64)
        dist.all_reduce(sent)
        if rank == 0:
            q.put(([[(int(p[0]) // 1000 if p.numel() else -1, p.numel(), float(p.sum())) for p in parts]
                    for parts in got], sent.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("lengths", [[300, 120, 250, 7, 199], [5000, 3, 2, 1], [64]])
def test_gather_waveforms_world2_gloo(lengths):
    """Uneven shards (and a rank with nothing): exactly the non-root ranks' samples travel, no padding."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, lengths, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, moved = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = shard_utterances(lengths, world)
    # bytes sent (all ranks) == bytes received at rank 0 == 4 x the samples of rank 1's utterances
    assert moved == [4 * sum(lengths[i] for i in shards[1])] * 2
    for r in range(world):
        assert len(res[r]) == len(shards[r])
        for (uid, n, s), i in zip(res[r], shards[r]):
            assert uid == i and n == lengths[i]
            assert s == pytest.approx(sum(range(lengths[i])) + 1000 * i * lengths[i])
