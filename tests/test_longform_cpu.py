"""One long utterance over ranks (rvc_amd.longform): the time-tile plan, and the sharded-by-time pass +
all_gather exchange against the whole-image pass on a finite-receptive-field stand-in for the U-Net,
world_size 2 and 3 over gloo on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from rvc_amd.longform import ALIGN, exchange_tiles, tile_plan


def test_tile_plan_covers_and_aligns():
    for Tp, world in ((32, 1), (3232, 2), (3232, 8), (96, 8), (360000 // 32 * 32, 8)):
        plan = tile_plan(Tp, world, halo=1024)
        assert plan[0][0] == 0 and plan[-1][1] == Tp
        for (a, b, r0, r1), nxt in zip(plan, plan[1:] + [None]):
            assert a % ALIGN == 0 and b % ALIGN == 0 and r0 % ALIGN == 0 and r1 % ALIGN == 0
            assert r0 == max(0, a - 1024) and r1 == min(Tp, b + 1024) and a <= b
            if nxt is not None:
                assert nxt[0] == b
        sizes = [b - a for a, b, _, _ in plan]
        assert max(sizes) - min(sizes) <= ALIGN
    with pytest.raises(ValueError):
        tile_plan(100, 2)


def _unet_standin(x):
    """A finite receptive field (radius 8 x 24 = 192 rows), zero padding at the image border, and 2x pooling
    + upsampling (alignment matters): the properties of the RMVPE U-Net the tiling relies on."""
    y = x[None]
    k = torch.tensor([[[0.25, 0.5, 0.25]]], dtype=x.dtype)
    for _ in range(3):
        for _ in range(8):
            y = F.conv1d(y.reshape(-1, 1, y.shape[-1]), k, padding=1).reshape(y.shape) + 0.1 * y
        y = F.avg_pool1d(y, 2)
        y = F.conv1d(y.reshape(-1, 1, y.shape[-1]), k, padding=1).reshape(y.shape)
        y = F.interpolate(y, scale_factor=2, mode="nearest")
    return y[0]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, Tp, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(5)
        img = torch.randn(4, Tp, generator=g, dtype=torch.float64)
        got = exchange_tiles(lambda r0, r1: _unet_standin(img[:, r0:r1]), 4, Tp, dist, "cpu", halo=256)
        if rank == 0:
            q.put(float((got - _unet_standin(img)).abs().max()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("world,Tp", [(2, 1024), (3, 2048)])
def test_exchange_tiles_matches_whole_pass(world, Tp):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, Tp, q)) for r in range(world)]
    for p in procs:
        p.start()
    err = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert err <= 1e-12
