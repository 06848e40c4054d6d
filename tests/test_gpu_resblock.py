"""Fused ResBlock pair (csrc/resblock.hip): one launch of y (+)= x + c2(lrelu(c1(lrelu(x), d))) against
the two-launch split-bf16 conv path it replaces (bit-identical: same k-order, passes and epilogue order)
and against a plain torch fp32 reference of residuals.py:22-44 (one pair)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rvc_amd import ops
from rvc_amd.ops import ACT_LRELU, Conv

pytestmark = pytest.mark.gpu
DEV = "cuda"


def make_pair(C, K, seed):
    g = torch.Generator().manual_seed(seed)
    s = 1.0 / np.sqrt(C * K)
    w1 = torch.randn(C, C, K, generator=g) * s
    w2 = torch.randn(C, C, K, generator=g) * s
    b1 = torch.randn(C, generator=g) * 0.1
    b2 = torch.randn(C, generator=g) * 0.1
    return (w1, b1, w2, b2), Conv(w1, b1, device=DEV), Conv(w2, b2, device=DEV)


def two_launch(x, c1, c2, K, d, y=None, accumulate=False):
    t1 = c1(x, pad=(K * d - d) // 2, dil=d, in_act=ACT_LRELU, in_slope=0.1)
    out = y if y is not None else torch.empty_like(x)
    c2(t1, pad=(K - 1) // 2, out=out, res=x, in_act=ACT_LRELU, in_slope=0.1, accumulate=accumulate)
    return out


def torch_ref(x, w, K, d):
    w1, b1, w2, b2 = w
    xt = F.conv1d(F.leaky_relu(x[None], 0.1), w1, b1, padding=(K * d - d) // 2, dilation=d)
    xt = F.conv1d(F.leaky_relu(xt, 0.1), w2, b2, padding=(K - 1) // 2)
    return (xt + x[None])[0]


@pytest.mark.parametrize("C", [32, 64, 128])
@pytest.mark.parametrize("K,d", [(3, 1), (3, 5), (7, 3), (11, 1), (11, 5)])
@pytest.mark.parametrize("precision", ["fp32x6", "bf16x3", "bf16"])
def test_fused_pair_bit_identical_to_two_launches(C, K, d, precision):
    """C = 128 (round 4): 2 row fragments per wave, residual read from x; at <= 2 split planes only (the 6-pass
    pair does not fit LDS), and against a two-launch form without split-K (its per-conv k-order)."""
    if C == 128 and precision == "fp32x6":
        pytest.skip("the 128-channel pair takes <= 2 split planes")
    w, c1, c2 = make_pair(C, K, seed=C * 100 + K * 10 + d)
    L = 5003  # several tiles and a partial one
    x = torch.randn(C, L, generator=torch.Generator().manual_seed(K + d)).to(DEV)
    with ops.precision(precision), ops.splitk_target(0):
        assert C == 128 or ops.resblock_fusable(c1, c2, d)
        ref = two_launch(x, c1, c2, K, d)
        y = torch.full_like(x, float("nan"))
        ops.resblock_pair(x, y, c1, c2, d, 0.1)
        acc0 = torch.randn(C, L, generator=torch.Generator().manual_seed(7)).to(DEV)
        ya, yb = acc0.clone(), acc0.clone()
        two_launch(x, c1, c2, K, d, y=ya, accumulate=True)
        ops.resblock_pair(x, yb, c1, c2, d, 0.1, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    assert torch.equal(ya, yb)
    if precision == "fp32x6":
        r = torch_ref(x.cpu(), w, K, d)
        err = (y.cpu() - r).abs().max().item()
        assert err <= 2e-5 * max(1.0, r.abs().max().item()), err


@pytest.mark.parametrize("L", [1, 7, 100, 239, 240, 241])
def test_fused_pair_short_and_edge_lengths(L):
    C, K, d = 32, 11, 5
    w, c1, c2 = make_pair(C, K, seed=5)
    x = torch.randn(C, L, generator=torch.Generator().manual_seed(L)).to(DEV)
    r = torch_ref(x.cpu(), w, K, d)
    for prec in ("fp32", "fp32x6"):  # the default (split-fp16 at k = 11) and the 6-pass split-bf16 pair
        with ops.precision(prec):
            y = torch.empty_like(x)
            ops.resblock_pair(x, y, c1, c2, d, 0.1)
            torch.cuda.synchronize()
            assert (y.cpu() - r).abs().max().item() <= 2e-5 * max(1.0, r.abs().max().item())
            if prec == "fp32x6":
                assert torch.equal(y, two_launch(x, c1, c2, K, d))


def test_fused_pair_rejects_bad_args():
    w, c1, c2 = make_pair(32, 3, seed=1)
    x = torch.randn(32, 100, device=DEV)
    with pytest.raises(ValueError):
        ops.resblock_pair(x, x, c1, c2, 1, 0.1)  # aliasing
    w16, c16a, c16b = make_pair(16, 3, seed=2)
    assert not ops.resblock_fusable(c16a, c16b, 1)
    x16 = torch.randn(16, 100, device=DEV)
    with pytest.raises(RuntimeError):
        ops.resblock_pair(x16, torch.empty_like(x16), c16a, c16b, 1, 0.1)


@pytest.mark.parametrize("C", [32, 64, 128])
@pytest.mark.parametrize("K,d", [(3, 1), (7, 3), (11, 5)])
@pytest.mark.parametrize("scale", [1.0, 1e-4, 1e4])
def test_fused_pair_f16x3(C, K, d, scale):
    """Split-fp16 fused pair: its T scale is per fused tile, so it is not bit-identical to the two-launch form
    (whose c1 output is scaled per conv tile); both within 2e-5 (relative to the output's max) of torch's fp32
    pair, at any input magnitude (the power-of-2 scales follow the data), plain and accumulating."""
    w, c1, c2 = make_pair(C, K, seed=C * 100 + K * 10 + d + 1)
    L = 5003
    x = (torch.randn(C, L, generator=torch.Generator().manual_seed(K + d + 1)) * scale).to(DEV)
    with ops.precision("f16x3"):
        assert C == 128 or ops.resblock_fusable(c1, c2, d)
        y = torch.full_like(x, float("nan"))
        ops.resblock_pair(x, y, c1, c2, d, 0.1)
        acc0 = (torch.randn(C, L, generator=torch.Generator().manual_seed(7)) * scale).to(DEV)
        yb = acc0.clone()
        ops.resblock_pair(x, yb, c1, c2, d, 0.1, accumulate=True)
        ref2 = two_launch(x, c1, c2, K, d)
    torch.cuda.synchronize()
    r = torch_ref(x.cpu(), w, K, d)
    tol = 2e-5 * r.abs().max().item()
    assert (y.cpu() - r).abs().max().item() <= tol
    assert (ref2.cpu() - r).abs().max().item() <= tol
    assert (yb.cpu() - (r + acc0.cpu())).abs().max().item() <= tol + 2e-6 * acc0.abs().max().item()


@pytest.mark.parametrize("C", [32, 64])
@pytest.mark.parametrize("K,d", [(3, 1), (7, 3), (11, 5)])
@pytest.mark.parametrize("L,B", [(5003, 1), (241, 1), (16, 1), (3001, 3)])
def test_fused_pair_outputs_through_lds_bit_identical(C, K, d, L, B):
    """Round 6: the split-fp16 pair's outputs go through LDS (over the tile's residual rows) and the loader waves store
    them during the next tile (rvc_resblock_set_ylds 1; 2: at C = 32 from two R buffers by tile parity, after the next
    tile's c1 barriers).  Same bits as the compute waves' own stores -- plain and accumulating, ragged last tile, fewer
    tiles than workgroups, batched clips."""
    w, c1, c2 = make_pair(C, K, seed=C + K + d + L)
    g = torch.Generator().manual_seed(L + B)
    x = torch.randn(B, C, L, generator=g).to(DEV)
    acc0 = torch.randn(B, C, L, generator=g).to(DEV)
    lib = ops._lib.load()
    outs = []
    prev = lib.rvc_resblock_set_wide64(0)  # the LDS output path is the narrow C = 64 geometry's
    for on in (0, 1, 2):
        lib.rvc_resblock_set_ylds(on)
        try:
            with ops.precision("f16x3"):
                y = torch.full_like(x, float("nan"))
                ops.resblock_pair(x if B > 1 else x[0], y if B > 1 else y[0], c1, c2, d, 0.1)
                ya = acc0.clone()
                ops.resblock_pair(x if B > 1 else x[0], ya if B > 1 else ya[0], c1, c2, d, 0.1, accumulate=True)
            torch.cuda.synchronize()
            outs.append((y.cpu(), ya.cpu()))
        finally:
            lib.rvc_resblock_set_ylds(-1)
    lib.rvc_resblock_set_wide64(prev)
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0]) and not torch.isnan(o[0]).any()
        assert torch.equal(outs[0][1], o[1])


@pytest.mark.parametrize("K,d", [(3, 1), (7, 3), (11, 5)])
@pytest.mark.parametrize("L,B", [(5003, 1), (1, 1), (239, 1), (240, 1), (241, 1), (481, 2), (3001, 3)])
@pytest.mark.parametrize("precision", ["fp32", "bf16x3", "bf16"])
def test_fused_pair_wide64(K, d, L, B, precision):
    """Round 6: the C = 64 pair with 2 row fragments per wave (240 outputs per tile, residual from x) against the narrow
    form (1 row fragment, 112 outputs) -- bit-identical at bf16x3 / bf16 (no tile scales), within split-fp16's 2e-5 of
    the fp32 reference at "fp32" (its power-of-2 tile scales follow the tile) -- plain and accumulating, ragged and
    single-column lengths, batched clips."""
    C = 64
    w, c1, c2 = make_pair(C, K, seed=K * 7 + d + L)
    g = torch.Generator().manual_seed(L * 3 + B)
    x = torch.randn(B, C, L, generator=g).to(DEV)
    acc0 = torch.randn(B, C, L, generator=g).to(DEV)
    lib = ops._lib.load()
    outs = []
    for wide in (0, 1):
        prev = lib.rvc_resblock_set_wide64(wide)
        try:
            with ops.precision(precision):
                y = torch.full_like(x, float("nan"))
                ops.resblock_pair(x if B > 1 else x[0], y if B > 1 else y[0], c1, c2, d, 0.1)
                ya = acc0.clone()
                ops.resblock_pair(x if B > 1 else x[0], ya if B > 1 else ya[0], c1, c2, d, 0.1, accumulate=True)
            torch.cuda.synchronize()
            outs.append((y.cpu(), ya.cpu()))
        finally:
            lib.rvc_resblock_set_wide64(prev)
    assert not torch.isnan(outs[1][0]).any()
    if precision == "fp32":
        for b in range(B):
            r = torch_ref(x[b].cpu(), w, K, d)
            tol = 2e-5 * max(1.0, r.abs().max().item())
            for o in outs:
                assert (o[0][b] - r).abs().max().item() <= tol
                assert (o[1][b] - (r + acc0[b].cpu())).abs().max().item() <= tol + 2e-6 * acc0.abs().max().item()
    else:
        assert torch.equal(outs[0][0], outs[1][0])
        assert torch.equal(outs[0][1], outs[1][1])
