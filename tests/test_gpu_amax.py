"""The |max| side channel (include/rvc_amd.h rvc_conv1d_args.amax_in / amax_out), pinned producer by producer.

A consumer in split-fp16 scales its activations by a power of 2 chosen from the cell its producer published; a cell
that under-reports max |y| would push the real peak past fp16's range (inf), so every producer form is checked to
publish EXACTLY max |y| of the tensor it wrote -- bit for bit, per batch element (round 6: one cell per element):
the conv engines' epilogues (bias2 / residual / accumulate / activation / polyphase store / ragged tails / batch / the
LDS tile epilogue / the fused source conv), the split-K reduce, the f32 engine, both LayerNorm forms, attention with
and without split-KV (its combine kernel), and ContentVec's fused layer 0.  Then a consumer whose input peak sits in the
last ragged tile, against torch f64 within test_conv1d_f16x3's bound.  Reference: the ResBlock chain whose activations
these cells carry, main/library/algorithm/residuals.py:36-44."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rvc_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def gen(seed):
    return torch.Generator().manual_seed(seed)


def assert_cell(cell, y, B):
    """cell (B cells) == max |y[b]| for every batch element, exactly."""
    y = y.reshape(B, -1)
    for b in range(B):
        want = float(y[b].abs().max().item())
        got = ops.amax_value(cell, b)
        assert got == want, (b, got, want)
        assert np.isfinite(got) and got > 0


@pytest.mark.parametrize("prec", ["fp32", "f16x3", "fp32x6", "bf16x3"])
@pytest.mark.parametrize("Ci,Co,K,d,L,B,epi", [
    (128, 128, 11, 5, 5003, 1, "rb"),     # the 128 x 256 split-fp16 tile, ragged last tile
    (64, 64, 5, 1, 3001, 2, "full"),      # bias2 / tanh / scale / residual / accumulate, batched, Lout % 4 != 0
    (40, 72, 3, 1, 777, 2, "full"),       # ragged rows and channels, batched
    (256, 256, 7, 1, 300, 1, "plain"),
    (32, 32, 3, 1, 4099, 3, "rb"),
])
@pytest.mark.parametrize("tile_epi", [0, 1])
def test_amax_conv_epilogue(prec, Ci, Co, K, d, L, B, epi, tile_epi):
    g = gen(Ci + K + B)
    x = torch.randn(B, Ci, L, generator=g).to(DEV)
    x[:, :, -1] *= 50.0  # the peak tends to the last (ragged) column
    w = torch.randn(Co, Ci, K, generator=g) / math.sqrt(Ci * K)
    c = ops.Conv(w, torch.randn(Co, generator=g))
    b2 = torch.randn(Co, generator=g).to(DEV)
    res = torch.randn(B, Co, L, generator=g).to(DEV)
    y = torch.randn(B, Co, L, generator=g).to(DEV) if epi == "full" else torch.empty(B, Co, L, device=DEV)
    kw = dict(pad=d * (K - 1) // 2, dil=d, out=y)
    if epi == "rb":
        kw.update(res=res, in_act=ops.ACT_LRELU, in_slope=0.1)
    elif epi == "full":
        kw.update(bias2=b2, res=res, accumulate=True, in_act=ops.ACT_LRELU, in_slope=0.1, in_scale=0.5,
                  out_act=ops.ACT_TANH, out_scale=-3.0)
    cells = ops.AmaxSlots(1, DEV, B)
    lib = ops._lib.load()
    lib.rvc_conv1d_set_tile_epi(tile_epi)
    try:
        with ops.precision(prec):
            c(x if B > 1 else x[0], amax_out=cells[0],
              **{k: (v[0] if B == 1 and torch.is_tensor(v) and v.dim() == 3 else v) for k, v in kw.items()})
        assert ops.LAST_CONV_ENGINE == 1
    finally:
        lib.rvc_conv1d_set_tile_epi(-1)
    torch.cuda.synchronize()
    assert_cell(cells[0], y, B)


@pytest.mark.parametrize("target", [0, 1 << 20])
@pytest.mark.parametrize("Ci,Co,K,L,B", [(768, 768, 1, 1599, 1), (192, 160, 3, 900, 2)])
def test_amax_splitk_reduce(Ci, Co, K, L, B, target):
    """target 1<<20 forces split-K: the partial tiles go to the workspace and conv_splitk_reduce stores and publishes."""
    g = gen(5)
    x = torch.randn(B, Ci, L, generator=g).to(DEV)
    c = ops.Conv(torch.randn(Co, Ci, K, generator=g) / math.sqrt(Ci * K), torch.randn(Co, generator=g))
    y = torch.randn(B, Co, L, generator=g).to(DEV)
    cells = ops.AmaxSlots(1, DEV, B)
    with ops.splitk_target(target):
        c(x if B > 1 else x[0], pad=(K - 1) // 2, out=y if B > 1 else y[0], accumulate=True, amax_out=cells[0])
    assert (ops.LAST_CONV_WS > 0) == (target > 0), ops.LAST_CONV_WS
    torch.cuda.synchronize()
    assert_cell(cells[0], y, B)


@pytest.mark.parametrize("case", [(1, 256, 80, 40, 20, 40 * 50, 1), (1, 128, 8, 4, 2, 4000, 2),
                                  (512, 512, 3, 2, 0, 1200, 1), (768, 768, 128, 1, 64, 300, 2)])
def test_amax_f32_engine(case):
    """The f32-MFMA engine's epilogue (strided, 1-channel and grouped convs: the feature extractor, pos_conv)."""
    Ci, Co, K, s, p, L, B = case
    groups = 16 if K == 128 else 1
    g = gen(K)
    old = ops.X6
    ops.X6 = False
    try:
        c = ops.Conv(torch.randn(Co, Ci // groups, K, generator=g) / math.sqrt(Ci // groups * K),
                     torch.randn(Co, generator=g), groups=groups)
    finally:
        ops.X6 = old
    x = torch.randn(B, Ci, L, generator=g).to(DEV)
    cells = ops.AmaxSlots(1, DEV, B)
    y = c(x if B > 1 else x[0], stride=s, pad=p, out_act=ops.ACT_GELU, amax_out=cells[0])
    assert ops.LAST_CONV_ENGINE == 0
    torch.cuda.synchronize()
    assert_cell(cells[0], y, B)


@pytest.mark.parametrize("C,T,B", [(768, 1599, 2), (512, 333, 1), (192, 3198, 2), (256, 100, 1)])
def test_amax_layernorm(C, T, B):
    """Both LayerNorm forms (the register form at 256 < C <= 768, the LDS tile form elsewhere) publish max |out|."""
    g = gen(C)
    x = torch.randn(B, C, T, generator=g).to(DEV)
    r = torch.randn(B, C, T, generator=g).to(DEV)
    gm = (torch.rand(C, generator=g) * 3).to(DEV)
    bt = torch.randn(C, generator=g).to(DEV)
    out = torch.empty(B, C, T, device=DEV)
    cells = ops.AmaxSlots(1, DEV, B)
    ops.layernorm_cf(x, r, gm, bt, out, B, C, T, amax_out=cells[0])
    torch.cuda.synchronize()
    assert_cell(cells[0], out, B)
    ref = F.layer_norm((x + r).transpose(1, 2), (C,), gm, bt, 1e-5).transpose(1, 2)
    assert (out - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("T,B,split", [(200, 2, False), (1600, 1, True), (640, 2, True)])
def test_amax_attention(T, B, split):
    """One key split (attn_fwd publishes) and split-KV (attn_combine publishes), batched and not."""
    H, D = 12, 64
    g = gen(T)
    qkv = torch.randn(B, 3 * H * D, T, generator=g).to(DEV)
    o = torch.empty(B, H * D, T, device=DEV)
    a = ops._lib.AttnArgs()
    a.B, a.H, a.D, a.T = B, H, D, T
    assert (ops._lib.load().rvc_attention_workspace_bytes(ctypes_ref(a)) > 0) == split, \
        "the shape no longer exercises the form it names"
    cells = ops.AmaxSlots(1, DEV, B)
    E = H * D
    ops.attention(qkv, qkv[:, E:], qkv[:, 2 * E:], o, B=B, H=H, D=D, T=T, ldc=T, q_hs=D * T, k_hs=D * T, v_hs=D * T,
                  o_hs=D * T, scale=D ** -0.5, q_bs=3 * E * T, k_bs=3 * E * T, v_bs=3 * E * T, o_bs=E * T,
                  amax_out=cells[0])
    torch.cuda.synchronize()
    assert_cell(cells[0], o, B)


def ctypes_ref(a):
    import ctypes
    return ctypes.byref(a)


@pytest.mark.parametrize("B,N", [(1, 16000 * 2 + 77), (2, 9000)])
def test_amax_fe0(B, N):
    g = gen(N)
    wav = torch.randn(B, N, generator=g) * 0.3
    c = ops.Conv(torch.randn(512, 1, 10, generator=g) * 0.3, None)
    gamma, beta = (torch.rand(512, generator=g) + 0.5).to(DEV), (torch.randn(512, generator=g) * 0.1).to(DEV)
    cells = ops.AmaxSlots(1, DEV, B)
    out = ops.fe0_gn_gelu(wav.to(DEV).contiguous(), c.w, gamma, beta, B, N, 512, 10, 5, amax_out=cells[0])
    torch.cuda.synchronize()
    assert_cell(cells[0], out, B)


@pytest.mark.parametrize("u,k,ci,co,L,B", [(12, 24, 64, 32, 300, 1), (10, 20, 256, 128, 200, 2), (2, 4, 64, 32, 2001, 1)])
@pytest.mark.parametrize("target", [-1, 1 << 20])
def test_fused_source_conv_bit_identical(u, k, ci, co, L, B, target):
    """ups(x) + noise_convs(har) in one call (rvc_conv1d_args.src_*, synthesizers.py:156) equals the upsampling
    conv followed by the separate 1-channel conv on the f32 engine with accumulate -- bit for bit (the source pass
    is that conv's fmaf chain) -- with and without split-K, and its published |max| is max |y| of the final values.
    Also against torch's fp32 ConvTranspose1d + Conv1d."""
    g = gen(u * k + B)
    x = torch.randn(B, ci, L, generator=g)
    w = torch.randn(ci, co, k, generator=g) / math.sqrt(ci * k / u)
    b = torch.randn(co, generator=g)
    p = (k - u) // 2
    up = ops.ConvT(w, b, u, p)
    Lout = up.out_len(L)
    stride_f0 = 4 if u != 2 else 1
    kn = 1 if stride_f0 == 1 else stride_f0 * 2 - stride_f0 % 2
    npad = 0 if stride_f0 == 1 else (kn - stride_f0) // 2
    Lh = Lout * stride_f0
    har = torch.randn(B, Lh, generator=g)
    wn, bn = torch.randn(co, 1, kn, generator=g) * 0.5, torch.randn(co, generator=g) * 0.1
    old = ops.X6
    ops.X6 = False
    try:
        nc_f32 = ops.Conv(wn, bn)
    finally:
        ops.X6 = old
    nc = ops.Conv(wn, bn)
    xd, hd = x.to(DEV), har.to(DEV)
    cells = ops.AmaxSlots(2, DEV, B)
    with ops.splitk_target(target if target >= 0 else None):
        y_sep = up(xd if B > 1 else xd[0], in_act=ops.ACT_LRELU, in_slope=0.1)
        nc_f32(hd.view(B, 1, Lh) if B > 1 else hd.view(1, Lh), Lout=Lout, stride=stride_f0, pad=npad, out=y_sep,
               accumulate=True, amax_out=cells[0])
        assert ops.LAST_CONV_ENGINE == 0
        y_fused = up(xd if B > 1 else xd[0], in_act=ops.ACT_LRELU, in_slope=0.1, src=(nc, hd, stride_f0, npad),
                     amax_out=cells[1])
    torch.cuda.synchronize()
    assert torch.equal(y_fused, y_sep), (y_fused - y_sep).abs().max().item()
    assert_cell(cells[1], y_fused, B)
    assert_cell(cells[0], y_sep, B)
    ref = F.conv_transpose1d(F.leaky_relu(x, 0.1), w, b, u, p) + F.conv1d(har.unsqueeze(1), wn, bn, stride_f0, npad)
    assert (y_fused.cpu().reshape(ref.shape) - ref).abs().max().item() <= 2e-5 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("Ci,Co,K,d,L", [(128, 128, 11, 5, 5003), (64, 64, 3, 1, 4099), (256, 256, 7, 3, 1777)])
def test_consumer_peak_in_last_ragged_tile(Ci, Co, K, d, L):
    """A producer (a K = 1 conv with an epilogue residual) writes x whose |max| -- 1e4 x the rest -- sits in the last,
    ragged column tile; it publishes the cell, and a split-fp16 consumer takes its scale from it: finite, and within
    test_conv1d_f16x3's bound of torch f64 (relative to the row's sum of |products|)."""
    g = gen(L)
    x0 = torch.randn(Ci, L, generator=g)
    x0[Ci // 3, L - 2] = 3.0e4
    prod = ops.Conv(torch.randn(Ci, Ci, 1, generator=g) * 1e-3, None)
    cells = ops.AmaxSlots(1, DEV)
    xd = prod(torch.randn(Ci, L, generator=g).to(DEV), res=x0.to(DEV), amax_out=cells[0])
    torch.cuda.synchronize()
    assert_cell(cells[0], xd, 1)
    assert int(xd.abs().argmax().item()) % L >= L - 256  # the peak is in the last 256-wide tile
    w = torch.randn(Co, Ci, K, generator=g) / math.sqrt(Ci * K)
    bb = torch.randn(Co, generator=g) * 0.1
    c = ops.Conv(w, bb)
    with ops.precision("f16x3"):
        y = c(xd, pad=d * (K - 1) // 2, dil=d, amax_in=cells[0], in_act=ops.ACT_LRELU, in_slope=0.1)
    assert ops.LAST_CONV_ENGINE == 1 and ops.LAST_CONV_PASSES == ops.F16X3
    y = y.cpu().double()
    assert torch.isfinite(y).all()
    xin = F.leaky_relu(xd.cpu().double(), 0.1)
    ref = F.conv1d(xin.unsqueeze(0), w.double(), bb.double(), 1, d * (K - 1) // 2, d)[0]
    mag = F.conv1d(xin.abs().unsqueeze(0), w.double().abs(), bb.double().abs(), 1, d * (K - 1) // 2, d)[0]
    f32 = F.conv1d(xin.float().unsqueeze(0), w, bb, 1, d * (K - 1) // 2, d)[0].double()
    rms = lambda e: e.pow(2).mean(1).sqrt() / mag.pow(2).mean(1).sqrt().clamp_min(1e-300)  # noqa: E731
    rel, rel32 = rms(y - ref), rms(f32 - ref)
    assert float(rel.max()) < 2.0 ** -18, float(rel.max())
    assert bool((rel <= 8 * rel32 + 1e-6).all()), (float(rel.max()), float(rel32.max()))


def _mha_ref64(q, k, v, H, D, T, scale):
    """softmax(q' k^T) v in f64 per head, q [B][H*D][T] -> [B][H*D][T]."""
    B = q.shape[0]
    qh = q.double().view(B, H, D, T).transpose(2, 3) * scale
    kh = k.double().view(B, H, D, T).transpose(2, 3)
    vh = v.double().view(B, H, D, T).transpose(2, 3)
    o = torch.softmax(qh @ kh.transpose(2, 3), -1) @ vh
    return o.transpose(2, 3).reshape(B, H * D, T)


@pytest.mark.parametrize("H,D,T,B", [(12, 64, 333, 1), (12, 64, 1599, 1), (12, 64, 640, 2), (2, 96, 257, 1),
                                     (2, 96, 3198, 1)])
def test_attention_split_f16(H, D, T, B):
    """The split-fp16 attention (rvc_attention_ex with the QKV projection's |max| cell): against torch f64, within 4x
    the f32-MFMA kernel's own error (+ 1e-6 of the output scale), and its |max| cell exact.  Covers one and several
    key splits, a ragged last key / query tile and batch."""
    g = gen(T + H)
    qkv = torch.randn(B, 3 * H * D, T, generator=g)
    qkv[:, :, T // 3] *= 8.0  # one loud frame
    E = H * D
    cell = ops.AmaxSlots(1, DEV, B)
    for b in range(B):
        cell.words[b * ops.AMAX_SHARDS] = int(np.float32(qkv[b].abs().max().item()).view(np.int32))
    dq = qkv.to(DEV)
    ref = _mha_ref64(qkv[:, :E], qkv[:, E:2 * E], qkv[:, 2 * E:], H, D, T, D ** -0.5)
    outs = {}
    for name, cin in (("f32", None), ("f16", cell[0])):
        o = torch.empty(B, E, T, device=DEV)
        oc = ops.AmaxSlots(1, DEV, B)
        ops.attention(dq, dq[:, E:], dq[:, 2 * E:], o, B=B, H=H, D=D, T=T, ldc=T, q_hs=D * T, k_hs=D * T, v_hs=D * T,
                      o_hs=D * T, scale=D ** -0.5, q_bs=3 * E * T, k_bs=3 * E * T, v_bs=3 * E * T, o_bs=E * T,
                      amax_in=cin, amax_out=oc[0])
        torch.cuda.synchronize()
        assert_cell(oc[0], o, B)
        outs[name] = o.cpu().double()
    e32 = (outs["f32"] - ref).abs().max().item()
    e16 = (outs["f16"] - ref).abs().max().item()
    assert e16 <= 4 * e32 + 1e-6 * ref.abs().max().item(), (e16, e32)
    assert not torch.equal(outs["f16"], outs["f32"])  # the split-fp16 kernel ran


def test_attention_split_f16_relpos_band():
    """The TextEncoder's rel-pos MHA (synthesizers.py:227-251) in split-fp16 vs the oracle's restatement."""
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
    ref = osy._mha(W, "a.", x, torch.ones(1, 1, T, T), H)[0]
    wqkv = torch.cat([W["a.conv_q.weight"], W["a.conv_k.weight"], W["a.conv_v.weight"]], 0)
    bqkv = torch.cat([W["a.conv_q.bias"], W["a.conv_k.bias"], W["a.conv_v.bias"]], 0)
    cell = ops.AmaxSlots(1, DEV)
    qkv = ops.Conv(wqkv, bqkv)(x[0].to(DEV), amax_out=cell[0])
    scale = 1 / math.sqrt(D)
    rk = ops.Conv(W["a.emb_rel_k"][0].unsqueeze(-1), None)(qkv, B=H, Lin=T, x_bstride=D * T, Lout=T, out_scale=scale)
    o = torch.empty(C, T, device=DEV)
    ml = torch.empty(H, 2, T, device=DEV)
    ops.attention(qkv, qkv[C:], qkv[2 * C:], o, B=1, H=H, D=D, T=T, ldc=T, q_hs=D * T, k_hs=D * T, v_hs=D * T,
                  o_hs=D * T, scale=scale, rk=rk, ev=W["a.emb_rel_v"][0].contiguous().to(DEV), ml=ml, W=10,
                  amax_in=cell[0])
    y = ops.Conv(W["a.conv_o.weight"], W["a.conv_o.bias"])(o).cpu()
    err = (y - ref).abs().max().item()
    assert err <= 1e-4 * max(1.0, ref.abs().max().item()), err
