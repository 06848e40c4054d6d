"""Op-level parity of the HIP kernels (through the C ABI) against torch-CPU fp32 references."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def gen(seed):
    return torch.Generator().manual_seed(seed)


def close(a, b, rtol=2e-5, atol=2e-5):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    assert a.shape == b.shape, (a.shape, b.shape)
    err = (a - b).abs().max().item()
    scale = b.abs().max().item()
    assert err <= atol + rtol * scale, f"max err {err} (scale {scale})"


@pytest.fixture(scope="module")
def ops():
    from rvc_amd import ops as o
    o._lib.load()
    return o


@pytest.fixture(params=[False, True], ids=["f32mfma", "x6"])
def engine(request, ops):
    """Run a conv test on the f32-MFMA engine and on the split-bf16 (x6) engine."""
    old = ops.X6
    ops.X6 = request.param
    yield request.param
    ops.X6 = old


CONV_CASES = [
    # Ci, Co, K, stride, dil, pad, groups, L
    (32, 32, 3, 1, 1, 1, 1, 5000),
    (32, 32, 11, 1, 5, 25, 1, 3000),
    (64, 64, 7, 1, 3, 9, 1, 2000),
    (128, 128, 3, 1, 1, 1, 1, 1500),
    (192, 768, 3, 1, 1, 1, 1, 700),
    (768, 192, 3, 1, 1, 1, 1, 700),
    (1, 256, 80, 40, 1, 20, 1, 40 * 50),
    (1, 512, 10, 5, 1, 0, 1, 4000),
    (512, 512, 3, 2, 1, 0, 1, 1200),
    (512, 512, 2, 2, 1, 0, 1, 800),
    (768, 768, 128, 1, 1, 64, 16, 300),
    (32, 1, 7, 1, 1, 3, 1, 3000),
    (192, 21, 1, 1, 1, 0, 1, 500),
    (256, 4608, 1, 1, 1, 0, 1, 1),
    (64, 64, 11, 1, 5, 25, 1, 4000),     # generator ResBlock shape (dilated)
    (40, 72, 3, 1, 1, 1, 1, 777),        # ragged channel chunks / fragments
    (40, 72, 3, 2, 1, 1, 1, 777),        # the same, stride 2 (split-bf16 strided staging)
    (768, 3072, 1, 1, 1, 0, 1, 1599),    # ContentVec fc1
    (256, 256, 7, 1, 1, 3, 1, 300),      # ragged N tile
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv1d(ops, engine, case):
    Ci, Co, K, s, d, p, g, L = case
    x = torch.randn(Ci, L, generator=gen(1))
    w = torch.randn(Co, Ci // g, K, generator=gen(2)) / math.sqrt(Ci // g * K)
    b = torch.randn(Co, generator=gen(3))
    ref = F.conv1d(x.unsqueeze(0), w, b, s, p, d, g)[0]
    c = ops.Conv(w, b, groups=g)
    y = c(x.to(DEV), stride=s, pad=p, dil=d)
    close(y, ref)


@pytest.mark.parametrize("case", [(768, 768, 128, 64, 16, 1599, 2, False), (768, 768, 128, 64, 16, 333, 1, True),
                                  (256, 256, 16, 8, 4, 1000, 2, True), (96, 96, 5, 2, 3, 777, 1, False)])
def test_conv1d_grouped_x6(ops, case):
    """Grouped convs on the split-operand engine, one group per phase (conv1d.hip gx6): ContentVec's pos_conv epilogue
    (GELU, + x, SamePad's dropped last column via Lout) over a clip batch, with and without the input's |max| cell
    (Cig = 64: the fast loader form), against torch fp32; the output cell holds max |y| per clip."""
    Ci, Co, K, p, g, L, B, cell_in = case
    x = torch.randn(B, Ci, L, generator=gen(30))
    w = torch.randn(Co, Ci // g, K, generator=gen(31)) / math.sqrt(Ci // g * K)
    b = torch.randn(Co, generator=gen(32)) * 0.1
    Lout = L
    ref = F.gelu(F.conv1d(x, w, b, 1, p, 1, g)[..., :Lout]) + x
    c = ops.Conv(w, b, groups=g)
    xd = x.to(DEV)
    cells = ops.AmaxSlots(2, DEV, B)
    if cell_in:
        cells[0].view(B, ops.AMAX_SHARDS)[:, 0] = torch.tensor(
            [float(x[i].abs().max()) for i in range(B)]).view(torch.int32).to(DEV)
    y = c(xd if B > 1 else xd[0], pad=p, Lout=Lout, out_act=ops.ACT_GELU, res=xd if B > 1 else xd[0],
          amax_in=cells[0] if cell_in else None, amax_out=cells[1])
    assert ops.LAST_CONV_ENGINE == 1 and ops.LAST_CONV_WS == 0
    close(y.view(B, Co, Lout), ref)
    torch.cuda.synchronize()
    for i in range(B):
        assert ops.amax_value(cells[1], i) == float(y.view(B, Co, Lout)[i].abs().max().cpu())


@pytest.mark.parametrize("prec,lo,hi", [("bf16x3", 0.0, 1e-4), ("bf16", 1e-4, 1e-2)])
@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[3] == 1 and c[6] == 1 and c[2] <= 16])
def test_conv1d_reduced_precision(ops, case, prec, lo, hi):
    """The split-bf16 engine at 3 passes (hH+hM+mH) and 1 pass (bf16 operands): relative RMS error vs the
    fp32 reference inside the band each arithmetic implies (the lower bound proves the mode is live)."""
    Ci, Co, K, s, d, p, g, L = case
    x = torch.randn(Ci, L, generator=gen(1))
    w = torch.randn(Co, Ci, K, generator=gen(2)) / math.sqrt(Ci * K)
    b = torch.randn(Co, generator=gen(3)) * 0.1
    ref = F.conv1d(x.unsqueeze(0).double(), w.double(), b.double(), s, p, d)[0]
    c = ops.Conv(w, b)
    with ops.precision(prec):
        y = c(x.to(DEV), stride=s, pad=p, dil=d)
    assert ops.LAST_CONV_ENGINE == 1
    rel = float(((y.cpu().double() - ref).pow(2).mean() / ref.pow(2).mean()).sqrt())
    assert lo <= rel < hi, rel


def test_conv1d_fused_epilogue(ops, engine):
    Ci, Co, K, L = 64, 64, 5, 3000
    x = torch.randn(Ci, L, generator=gen(4))
    w = torch.randn(Co, Ci, K, generator=gen(5)) / math.sqrt(Ci * K)
    b = torch.randn(Co, generator=gen(6))
    b2 = torch.randn(Co, generator=gen(7))
    res = torch.randn(Co, L, generator=gen(8))
    acc0 = torch.randn(Co, L, generator=gen(9))
    pre = F.leaky_relu(x * (1 / 3), 0.1)
    ref = acc0 + (torch.tanh(F.conv1d(pre.unsqueeze(0), w, b, 1, 2)[0] + b2[:, None]) * -1.0 + res)
    c = ops.Conv(w, b)
    y = acc0.to(DEV)
    c(x.to(DEV), pad=2, bias2=b2.to(DEV), res=res.to(DEV), out=y, accumulate=True, in_act=ops.ACT_LRELU,
      in_slope=0.1, in_scale=1 / 3, out_act=ops.ACT_TANH, out_scale=-1.0)
    close(y, ref)


@pytest.mark.parametrize("u,k,ci,co,L", [(12, 24, 64, 32, 300), (10, 20, 64, 32, 300), (10, 16, 64, 32, 200),
                                          (2, 4, 32, 16, 2000), (8, 16, 64, 32, 100)])
def test_conv_transpose(ops, engine, u, k, ci, co, L):
    x = torch.randn(ci, L, generator=gen(10))
    w = torch.randn(ci, co, k, generator=gen(11)) / math.sqrt(ci * k / u)
    b = torch.randn(co, generator=gen(12))
    p = (k - u) // 2
    ref = F.conv_transpose1d(F.leaky_relu(x, 0.1).unsqueeze(0), w, b, u, p)[0]
    c = ops.ConvT(w, b, u, p)
    y = c(x.to(DEV), in_act=ops.ACT_LRELU, in_slope=0.1)
    close(y, ref)


@pytest.mark.parametrize("H,D,T", [(12, 64, 333), (12, 64, 1600), (2, 96, 257)])
def test_attention_plain(ops, H, D, T):
    q = torch.randn(H * D, T, generator=gen(20))
    k = torch.randn(H * D, T, generator=gen(21))
    v = torch.randn(H * D, T, generator=gen(22))
    scale = D ** -0.5
    qh = q.view(H, D, T).transpose(1, 2) * scale
    kh = k.view(H, D, T).transpose(1, 2)
    vh = v.view(H, D, T).transpose(1, 2)
    ref = torch.softmax(qh @ kh.transpose(1, 2), -1) @ vh  # [H, T, D]
    ref = ref.transpose(1, 2).reshape(H * D, T)
    o = torch.empty(H * D, T, device=DEV)
    ops.attention(q.to(DEV), k.to(DEV), v.to(DEV), o, B=1, H=H, D=D, T=T, ldc=T, q_hs=D * T, k_hs=D * T,
                  v_hs=D * T, o_hs=D * T, scale=scale)
    close(o, ref, rtol=1e-4, atol=1e-5)


def test_attention_relpos_band(ops):
    """TextEncoder rel-pos MHA vs the oracle's restatement (synthesizers.py:227-251)."""
    from oracle import synth as osy
    H, D, T = 2, 96, 300
    C = H * D
    W = {}
    g = gen(30)
    x = torch.randn(1, C, T, generator=g)
    for n in ("q", "k", "v", "o"):
        W[f"a.conv_{n}.weight"] = torch.randn(C, C, 1, generator=g) / math.sqrt(C)
        W[f"a.conv_{n}.bias"] = torch.randn(C, generator=g) * 0.1
    W["a.emb_rel_k"] = torch.randn(1, 21, D, generator=g) * D ** -0.5
    W["a.emb_rel_v"] = torch.randn(1, 21, D, generator=g) * D ** -0.5
    mask = torch.ones(1, 1, T, T)
    ref = osy._mha(W, "a.", x, mask, H)[0]
    wqkv = torch.cat([W["a.conv_q.weight"], W["a.conv_k.weight"], W["a.conv_v.weight"]], 0)
    bqkv = torch.cat([W["a.conv_q.bias"], W["a.conv_k.bias"], W["a.conv_v.bias"]], 0)
    qkv = ops.Conv(wqkv, bqkv)(x[0].to(DEV))
    scale = 1 / math.sqrt(D)
    rk = ops.Conv(W["a.emb_rel_k"][0].unsqueeze(-1), None)(qkv, B=H, Lin=T, x_bstride=D * T, Lout=T, out_scale=scale)
    o = torch.empty(C, T, device=DEV)
    ml = torch.empty(H, 2, T, device=DEV)
    ops.attention(qkv, qkv[C:], qkv[2 * C:], o, B=1, H=H, D=D, T=T, ldc=T, q_hs=D * T, k_hs=D * T, v_hs=D * T,
                  o_hs=D * T, scale=scale, rk=rk, ev=W["a.emb_rel_v"][0].contiguous().to(DEV), ml=ml, W=10)
    y = ops.Conv(W["a.conv_o.weight"], W["a.conv_o.bias"])(o)
    close(y, ref, rtol=1e-4, atol=1e-5)


def test_layernorm_gate_flip_transpose(ops):
    C, T = 192, 1000
    x = torch.randn(C, T, generator=gen(40))
    r = torch.randn(C, T, generator=gen(41))
    gm = torch.rand(C, generator=gen(42)) + 0.5
    bt = torch.randn(C, generator=gen(43))
    ref = F.layer_norm((x + r).t(), (C,), gm, bt, 1e-5).t()
    out = torch.empty(C, T, device=DEV)
    ops.layernorm_cf(x.to(DEV), r.to(DEV), gm.to(DEV), bt.to(DEV), out, 1, C, T)
    close(out, ref)
    a = torch.randn(2 * C, T, generator=gen(44))
    out = torch.empty(C, T, device=DEV)
    ops.gate(a.to(DEV), out, 1, C, T)
    close(out, torch.tanh(a[:C]) * torch.sigmoid(a[C:]))
    out = torch.empty(C, T, device=DEV)
    ops.flip_channels(x.to(DEV), out, 1, C, T)
    close(out, torch.flip(x, [0]), 0, 0)
    xt = torch.randn(777, 129, generator=gen(45))
    out = torch.empty(129, 777, device=DEV)
    ops.transpose(xt.to(DEV), out, 1, 777, 129)
    close(out, xt.t(), 0, 0)


@pytest.mark.parametrize("sr,upp,T", [(48000, 480, 400), (40000, 400, 2500), (32000, 320, 4100)])
def test_sine_source_matches_oracle(ops, sr, upp, T):
    from oracle import synth as osy
    f0 = (torch.rand(1, T, generator=gen(50)) * 1200).float()
    f0[:, torch.rand(T, generator=gen(51)) < 0.2] = 0
    noise = torch.randn(1, T * upp, 1, generator=gen(52))
    W = {"dec.m_source.l_linear.weight": torch.tensor([[0.9]]), "dec.m_source.l_linear.bias": torch.tensor([0.01])}
    ref = osy.sine_source(W, f0, upp, sr, noise)[0, 0]
    har = torch.empty(T * upp, device=DEV)
    work = torch.empty(T, device=DEV)
    ops.sine_source(f0.to(DEV), noise.to(DEV).view(-1), har, work, 1, T, upp, float(sr), 0.9, 0.01)
    close(har, ref, rtol=0, atol=2e-5)


def test_randn_moments(ops):
    out = torch.empty(1 << 20, device=DEV)
    ops.randn(out, seed=123)
    x = out.cpu().double()
    assert abs(x.mean().item()) < 5e-3 and abs(x.std().item() - 1) < 5e-3
    out2 = torch.empty(1 << 20, device=DEV)
    ops.randn(out2, seed=123)
    assert torch.equal(out.cpu(), out2.cpu())


@pytest.mark.parametrize("N,tpad", [(480000, 16000), (3001, 1000), (40, 0)])
def test_filtfilt_pad_matches_scipy(ops, N, tpad):
    """convert.py:403,416: scipy filtfilt (f64, odd padding) + reflect pad, on the device.

    Tolerance: the chunked recurrence reproduces scipy's sequential result up to rounding noise
    amplified by the filter's 1.7e7 transient state gain (~1e-7 of full scale)."""
    from scipy import signal
    from rvc_amd.pipeline import AH, BH
    x = (np.random.default_rng(N).standard_normal(N) * 0.3).astype(np.float32)
    ref = np.pad(signal.filtfilt(BH, AH, x), (tpad, tpad), mode="reflect")
    f = ops.FiltFilt(BH, AH)
    out, out64 = f(torch.from_numpy(x).to(DEV), tpad, want_f64=True)
    scale = np.abs(ref).max()
    np.testing.assert_allclose(out64.cpu().numpy(), ref, rtol=0, atol=1e-6 * scale)
    assert np.max(np.abs(out.cpu().numpy() - ref.astype(np.float32))) <= 1e-6 * scale
    assert np.sqrt(np.mean((out64.cpu().numpy() - ref) ** 2)) < 1e-7 * scale


def test_filtfilt_golden(ops, golden):
    """The reference's own filtfilt output (tests/golden/filtfilt.npz, f64 input) -- via f32, as the pipeline."""
    from scipy import signal
    from rvc_amd.pipeline import AH, BH
    g = golden("filtfilt")
    np.testing.assert_allclose(signal.filtfilt(BH, AH, g["x"]), g["y"], rtol=0, atol=1e-12)
    f = ops.FiltFilt(BH, AH)
    _, out64 = f(torch.from_numpy(g["x"].astype(np.float32)).to(DEV), 0, want_f64=True)
    np.testing.assert_allclose(out64.cpu().numpy(), g["y"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("f64", [False, True])
@pytest.mark.parametrize("Ci,Co,H,W", [(32, 32, 40, 24), (256, 256, 12, 8), (16, 16, 30, 20)])
def test_conv2d_bordered_image_writes_zero_border(ops, engine, Ci, Co, H, W, f64):
    """RMVPE's 3x3 conv on a zero-bordered [C][H+2][W+2] image (1-D engine, 9 tap offsets; the f32 engines and
    the f64 one of the f64 RMVPE): the interior matches F.conv2d(pad 1) and the border is written as exactly 0,
    so the output buffer needs no zero-fill (the 256-channel case runs split-K, whose reduce stores the border)."""
    from rvc_amd.rmvpe import _Conv2d
    if f64 and engine != "x6":
        pytest.skip("one engine for f64")
    g = gen(11)
    w = torch.randn(Co, Ci, 3, 3, generator=g, dtype=torch.float64) / math.sqrt(9 * Ci)
    b = torch.randn(Co, generator=g, dtype=torch.float64) * 0.1
    x = torch.randn(Ci, H, W, generator=g, dtype=torch.float64)
    dt = torch.float64 if f64 else torch.float32
    xb = F.pad(x.to(dt), (1, 1, 1, 1))
    conv = _Conv2d(w if f64 else w.float(), b if f64 else b.float(), DEV, f64=f64)
    out = torch.full((Co, H + 2, W + 2), float("nan"), device=DEV, dtype=dt)
    conv(xb.to(DEV).contiguous(), H, W, out)
    torch.cuda.synchronize()
    o = out.cpu()
    ref = F.conv2d(x.to(dt).double().unsqueeze(0), w.to(dt).double(), b.to(dt).double(), padding=1)[0]
    if f64:
        assert (o[:, 1:-1, 1:-1] - ref).abs().max().item() <= 1e-13 * max(1.0, ref.abs().max().item())
    else:
        close(o[:, 1:-1, 1:-1], ref)
    border = torch.ones(H + 2, W + 2, dtype=torch.bool)
    border[1:-1, 1:-1] = False
    assert torch.equal(o[:, border], torch.zeros(Co, int(border.sum())))


@pytest.mark.parametrize("Ci,Co,H,W,B,k", [(64, 128, 9, 4, 1, 3), (24, 40, 7, 5, 2, 3), (16, 16, 11, 3, 1, 3),
                                           (48, 72, 6, 4, 2, 1)])
def test_conv64_every_plan(ops, Ci, Co, H, W, B, k):
    """The f64 conv engine under every plan its planner can choose (rvc_conv64_set_plan: the 18 tiles, split-K
    1..8, bordered and compact forms -- the compact one's GEMM columns are the H x W interior cells, and its
    epilogue writes the border cells beside the image's edge cells): interior = F.conv2d in f64 to 1e-13, border
    exactly 0, over a NaN-filled output, batched (batch strides) and not."""
    g = gen(12)
    w = torch.randn(Co, Ci, k, k, generator=g, dtype=torch.float64) / math.sqrt(k * k * Ci)
    b = torch.randn(Co, generator=g, dtype=torch.float64) * 0.1
    x = torch.randn(B, Ci, H, W, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, w, b, padding=k // 2)
    wrap = W + 2
    L = (H + 2) * wrap
    toff = [dy * wrap + dx for dy in range(k) for dx in range(k)]
    wkm = ops.pack_km(w.reshape(Co, Ci, k * k)).to(DEV)
    xb = F.pad(x, (1, 1, 1, 1)).to(DEV).contiguous()
    border = torch.ones(H + 2, W + 2, dtype=torch.bool)
    border[1:-1, 1:-1] = False
    seen = set()
    try:
        for tile in range(18):
            for cmp in (0, 1):
                for ks in (1, 2, 3, 8):
                    try:
                        ops.conv64_set_plan(tile, ks, cmp)
                        out = torch.full((B, Co, H + 2, W + 2), float("nan"), device=DEV, dtype=torch.float64)
                        kw = dict(bias=b.to(DEV), pad=(wrap + 1) if k == 3 else 0, Lin=L, Lout=L, toff=toff,
                                  wrap=wrap, B=B, x_bstride=Ci * L, y_bstride=Co * L)
                        plan = ops.conv64(xb, wkm, Ci, Co, k * k, out=out, plan=True, **kw)
                        ops.conv64(xb, wkm, Ci, Co, k * k, out=out, **kw)
                    except RuntimeError:
                        continue  # a plan the planner refuses for this shape (staging budget / split count)
                    torch.cuda.synchronize()
                    seen.add(tuple(plan[:3]))
                    o = out.cpu()
                    err = (o[:, :, 1:-1, 1:-1] - ref).abs().max().item()
                    assert err <= 1e-13 * max(1.0, ref.abs().max().item()), (plan, err)
                    assert torch.equal(o[:, :, border], torch.zeros(B, Co, int(border.sum()), dtype=o.dtype)), plan
    finally:
        ops.conv64_set_plan()
    # (a K = 1 chunk stages 16 channel rows: only the narrower tiles fit it, and 3 chunks allow no split)
    assert len({p[0] for p in seen}) >= (6 if k == 3 else 4) and {p[2] for p in seen} == {0, 1}, seen
    assert k == 1 or max(p[1] for p in seen) >= 3, seen


@pytest.mark.parametrize("Ci,Co,H,W,B", [(64, 64, 12, 8, 1), (128, 96, 10, 4, 2), (72, 64, 9, 5, 1), (512, 512, 94, 4, 1),
                                         (16, 16, 12, 8, 1), (32, 16, 9, 5, 2), (64, 32, 10, 6, 1), (16, 32, 7, 4, 1),
                                         (32, 32, 33, 17, 1), (64, 16, 6, 70, 1)])
def test_wino64_conv(ops, Ci, Co, H, W, B):
    """The f64 Winograd F(4x4, 3x3) conv of RMVPE (rmvpe64.hip): for >= 64 channels the input transform, 36 GEMMs
    on the conv engine with per-batch weights and the output transform; for 16 / 32 / 64 -> 16 / 32 channels the
    fused kernel (transforms in LDS) -- each with bias, ReLU, residual and the zero border, against F.conv2d in
    f64 (1e-12 relative: the transforms cost ~1e-14) over a NaN-filled output, ragged tiles (H, W not multiples
    of 4) and batch strides included."""
    g = gen(13)
    w = torch.randn(Co, Ci, 3, 3, generator=g, dtype=torch.float64) / math.sqrt(9 * Ci)
    b = torch.randn(Co, generator=g, dtype=torch.float64) * 0.1
    x = torch.randn(B, Ci, H, W, generator=g, dtype=torch.float64)
    r = torch.randn(B, Co, H, W, generator=g, dtype=torch.float64)
    ref = torch.relu(F.conv2d(x, w, b, padding=1)) + r
    wkm = ops.pack_km(w.reshape(Co, Ci, 9)).to(DEV)
    v = ops.wino64_weights(wkm, Ci, Co)
    xb = F.pad(x, (1, 1, 1, 1)).to(DEV).contiguous()
    rb = F.pad(r, (1, 1, 1, 1)).to(DEV).contiguous()
    L = (H + 2) * (W + 2)
    out = torch.full((B, Co, H + 2, W + 2), float("nan"), device=DEV, dtype=torch.float64)
    ops.wino64(xb, v, Ci, Co, H, W, bias=b.to(DEV), res=rb, out=out, out_act=ops.ACT_RELU, B=B, x_bstride=Ci * L,
               y_bstride=Co * L, res_bstride=Co * L)
    torch.cuda.synchronize()
    o = out.cpu()
    err = (o[:, :, 1:-1, 1:-1] - ref).abs().max().item()
    assert err <= 1e-12 * max(1.0, ref.abs().max().item()), err
    border = torch.ones(H + 2, W + 2, dtype=torch.bool)
    border[1:-1, 1:-1] = False
    assert torch.equal(o[:, :, border], torch.zeros(B, Co, int(border.sum()), dtype=o.dtype))
    assert ops.wino64_use(Ci, Co) == (Ci >= 64 and Co >= 64)  # the fused small-channel form: tested, off by default
    if Ci >= 64 and Co >= 64:
        assert not ops.wino64_use(Ci, Co, 94, 4) and ops.wino64_use(Ci, Co, 188, 8)


F16_CASES = [c for c in CONV_CASES if c[6] == 1 and c[2] <= 64 and (c[3] == 1 or (c[3] == 2 and c[0] >= 32))]


@pytest.mark.parametrize("case", F16_CASES)
@pytest.mark.parametrize("spread", ["unit", "wide"])
def test_conv1d_f16x3(ops, case, spread):
    """Split-fp16 (3 fp16 MFMA passes over power-of-2-scaled 22-bit operands): error vs an f64 reference, per
    output row, measured against the row's sum of |products| (conv(|x|, |w|): the scale of any floating-point
    conv's error): below 2^-18 of it, and of the order of torch's own f32 conv error (<= 8x + 1e-6 of it),
    also when channels span 1e-6..1e6 ("wide": the per-tile activation and per-row weight scales must keep
    the small ones)."""
    Ci, Co, K, s, d, p, g, L = case
    x = torch.randn(Ci, L, generator=gen(11))
    w = torch.randn(Co, Ci, K, generator=gen(12)) / math.sqrt(Ci * K)
    b = torch.randn(Co, generator=gen(13)) * 0.1
    if spread == "wide":
        x = x * torch.logspace(-6, 6, Ci).unsqueeze(1)
        w = w * torch.logspace(3, -3, Co).view(Co, 1, 1)
    ref = F.conv1d(x.unsqueeze(0).double(), w.double(), b.double(), s, p, d)[0]
    mag = F.conv1d(x.unsqueeze(0).double().abs(), w.double().abs(), b.double().abs(), s, p, d)[0]
    f32 = F.conv1d(x.unsqueeze(0), w, b, s, p, d)[0].double()
    c = ops.Conv(w, b)
    with ops.precision("f16x3"):
        y = c(x.to(DEV), stride=s, pad=p, dil=d)
    assert ops.LAST_CONV_ENGINE == 1
    y = y.cpu().double()
    # per output row (rows differ by up to 1e6 in scale under "wide")
    rms = lambda e: e.pow(2).mean(1).sqrt() / mag.pow(2).mean(1).sqrt().clamp_min(1e-300)  # noqa: E731
    rel, rel32 = rms(y - ref), rms(f32 - ref)
    assert float(rel.max()) < 2.0 ** -18, float(rel.max())
    assert bool((rel <= 8 * rel32 + 1e-6).all()), (float(rel.max()), float(rel32.max()))


@pytest.mark.parametrize("prec", ["fp32", "fp32x6", "bf16x3"])
@pytest.mark.parametrize("Ci,Co,K,d,L,B,epi", [
    (128, 128, 11, 5, 5000, 1, "rb"),     # the 128 x 256 split-fp16 tile, ragged last tile
    (128, 128, 3, 1, 4096, 1, "rb"),      # full tiles, Lout % 4 == 0: the 16-B path everywhere
    (64, 64, 5, 1, 3001, 2, "full"),      # bias2 / tanh / scale / residual / accumulate, batched, Lout % 4 != 0
    (768, 768, 1, 1, 1599, 1, "plain"),   # split-K partial tiles through the workspace
    (40, 72, 3, 1, 777, 1, "full"),       # ragged rows and channels
    (256, 256, 7, 1, 300, 1, "rb"),
])
def test_x6_tile_epilogue_bit_identical(ops, prec, Ci, Co, K, d, L, B, epi):
    """The x6 engine's LDS tile epilogue (round 5) gives the same bits as the in-register epilogue it replaced, for
    every epilogue feature and tile shape (rvc_conv1d_set_tile_epi toggles it within the process)."""
    g = gen(11)
    x = torch.randn(B, Ci, L, generator=g).to(DEV)
    w = torch.randn(Co, Ci, K, generator=g) / math.sqrt(Ci * K)
    b = torch.randn(Co, generator=g)
    b2 = torch.randn(Co, generator=g).to(DEV)
    res = torch.randn(B, Co, L, generator=g).to(DEV)
    acc0 = torch.randn(B, Co, L, generator=g).to(DEV)
    c = ops.Conv(w, b)
    p = d * (K - 1) // 2
    outs = []
    lib = ops._lib.load()
    for on in (0, 1):
        lib.rvc_conv1d_set_tile_epi(on)
        try:
            y = acc0.clone() if epi == "full" else torch.empty(B, Co, L, device=DEV)
            kw = dict(pad=p, dil=d, out=y)
            if epi == "rb":
                kw.update(res=res, in_act=ops.ACT_LRELU, in_slope=0.1)
            elif epi == "full":
                kw.update(bias2=b2, res=res, accumulate=True, in_act=ops.ACT_LRELU, in_slope=0.1, in_scale=0.5,
                          out_act=ops.ACT_TANH, out_scale=-1.0)
            with ops.precision(prec):
                c(x if B > 1 else x[0], **{k: (v[0] if B == 1 and torch.is_tensor(v) and v.dim() == 3 else v)
                                           for k, v in kw.items()})
            assert ops.LAST_CONV_ENGINE == 1
            torch.cuda.synchronize()
            outs.append(y.cpu())
        finally:
            lib.rvc_conv1d_set_tile_epi(-1)
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max()


@pytest.mark.parametrize("Ci,Co,K,d,L,act", [(128, 128, 11, 5, 40000, "lrelu"), (128, 128, 3, 1, 33333, "none"),
                                             (256, 256, 7, 3, 9000, "lrelu"), (192, 160, 3, 1, 5000, "lrelu")])
def test_x6_f16_fast_loader_bit_identical(ops, Ci, Co, K, d, L, act):
    """The split-fp16 loaders' fast form (its own kernel, taken with the producer's |max| on the 8-compute-wave tiles)
    stages the same fp16 pieces as the general form: same bits (rvc_conv1d_set_f16_fast toggles it)."""
    g = gen(12)
    x = torch.randn(Ci, L, generator=g).to(DEV)
    w = torch.randn(Co, Ci, K, generator=g) / math.sqrt(Ci * K)
    c = ops.Conv(w, torch.randn(Co, generator=g))
    res = torch.randn(Co, L, generator=g).to(DEV)
    cell = ops.AmaxSlots(1, DEV)
    cell.words[0] = int(np.float32(x.abs().max().item()).view(np.int32))
    lib = ops._lib.load()
    outs = []
    for on in (0, 1):
        lib.rvc_conv1d_set_f16_fast(on)
        try:
            kw = dict(pad=d * (K - 1) // 2, dil=d, res=res, amax_in=cell[0])
            if act == "lrelu":
                kw.update(in_act=ops.ACT_LRELU, in_slope=0.1)
            with ops.precision("f16x3"):
                y = c(x, **kw)
            assert ops.LAST_CONV_ENGINE == 1
            torch.cuda.synchronize()
            outs.append(y.cpu())
        finally:
            lib.rvc_conv1d_set_f16_fast(-1)
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max()


@pytest.mark.parametrize("B,N,C,K,S", [(1, 16000 * 3 + 123, 512, 10, 5), (2, 8000, 512, 10, 5), (1, 400, 512, 10, 5),
                                       (1, 9001, 4096, 16, 8), (2, 3000, 100, 3, 1)])
def test_fe0_gn_gelu(ops, B, N, C, K, S):
    """ContentVec's first layer fused (rvc_fe0_gn_gelu: conv 1 -> 512, k10 s5, GroupNorm(512, 512), GELU) against
    torch's f64 evaluation of the reference's layers (fairseq.py:1165-1195); and at the entry's limits (the widest
    layer, K = 16 taps, stride 8; a ragged last channel group)."""
    g = gen(21)
    wav = torch.randn(B, N, generator=g) * 0.3
    w = torch.randn(C, 1, K, generator=g) * 0.3
    gamma, beta = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.1
    y = F.conv1d(wav.double().unsqueeze(1), w.double(), None, S)
    ref = F.gelu(F.group_norm(y, C, gamma.double(), beta.double(), 1e-5))
    c = ops.Conv(w, None)
    out = ops.fe0_gn_gelu(wav.to(DEV).contiguous(), c.w, gamma.to(DEV), beta.to(DEV), B, N, C, K, S)
    got = out.cpu().double().reshape(ref.shape)
    assert (got - ref).abs().max().item() < 2e-5 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("prec", ["fp32", "fp32x6", "bf16x3", "bf16"])
@pytest.mark.parametrize("case", [
    ("rb", 128, 128, 11, 5, 5003, 1),      # the 128 x 256 split-fp16 tile, ragged last tile
    ("full", 64, 64, 5, 1, 3001, 2),       # bias2 / tanh / scale / residual / accumulate, batched, Lout % 4 != 0
    ("full", 40, 72, 3, 1, 777, 1),        # ragged rows and channels
    ("rb", 256, 256, 7, 1, 300, 1),
    ("rb", 32, 32, 3, 1, 4099, 3),         # 32 x 128 tiles, batched
    ("convT", 64, 32, 12, 0, 300, 1),      # polyphase stores (ConvTranspose u = 12)
    ("convT", 256, 128, 10, 0, 200, 2),
])
def test_x6_epilogue_128b_rows_bit_identical(ops, prec, case):
    """The x6 engine's in-register epilogue in 128-byte rows (round 6, rvc_conv1d_set_swz: a v_permlane16_swap per
    accumulator pair of adjacent column fragments) gives the same bits as the 16-column form, for every epilogue feature,
    polyphase stores and batched launches."""
    epi, Ci, Co, K, d, L, B = case
    g = gen(Ci + Co + K)
    outs = []
    lib = ops._lib.load()
    if epi == "convT":
        u = K
        w = torch.randn(Ci, Co, 2 * u, generator=g) / math.sqrt(Ci * 2)
        c = ops.ConvT(w, torch.randn(Co, generator=g), u, u // 2)
        x = torch.randn(B, Ci, L, generator=g).to(DEV)
    else:
        w = torch.randn(Co, Ci, K, generator=g) / math.sqrt(Ci * K)
        c = ops.Conv(w, torch.randn(Co, generator=g))
        x = torch.randn(B, Ci, L, generator=g).to(DEV)
        b2 = torch.randn(Co, generator=g).to(DEV)
        res = torch.randn(B, Co, L, generator=g).to(DEV)
        acc0 = torch.randn(B, Co, L, generator=g).to(DEV)
    for on in (0, 1):
        lib.rvc_conv1d_set_swz(on)
        try:
            with ops.precision(prec), ops.splitk_target(0):
                if epi == "convT":
                    y = c(x if B > 1 else x[0], in_act=ops.ACT_LRELU, in_slope=0.1)
                else:
                    y = acc0.clone() if epi == "full" else torch.empty(B, Co, L, device=DEV)
                    kw = dict(pad=d * (K - 1) // 2, dil=d, out=y if B > 1 else y[0], res=res if B > 1 else res[0],
                              in_act=ops.ACT_LRELU, in_slope=0.1)
                    if epi == "full":
                        kw.update(bias2=b2, accumulate=True, in_scale=0.5, out_act=ops.ACT_TANH, out_scale=-1.0)
                    c(x if B > 1 else x[0], **kw)
                assert ops.LAST_CONV_ENGINE == 1
            torch.cuda.synchronize()
            outs.append(y.cpu())
        finally:
            lib.rvc_conv1d_set_swz(-1)
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max()
