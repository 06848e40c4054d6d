"""Tensor-level wrappers over the C ABI (torch tensors are only device buffers + streams here).

Every function checks shapes on the host before launching (a kernel that reads out
of bounds can reset the GPU), passes raw pointers, and raises on a non-zero status.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from . import _lib
from ._lib import ACT_GELU, ACT_LOGCLAMP, ACT_LRELU, ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_TANH, check  # noqa: F401


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    if t is None:
        return None
    if not t.is_cuda or t.dtype not in (torch.float32, torch.int64, torch.int32):
        raise TypeError(f"rvc_amd: expected a CUDA f32/int tensor, got {t.dtype} on {t.device}")
    return ctypes.c_void_p(t.data_ptr())


# ------------------------------------------------------------------ weight packing (host, load time)
def pack_km(w: torch.Tensor, groups: int = 1) -> torch.Tensor:
    """Conv weight [Co, Ci/g, K] -> KM layout [g][Ci/g*K][Co/g] (k = c*K + tap, m contiguous)."""
    Co, Cig, K = w.shape
    Cog = Co // groups
    return w.reshape(groups, Cog, Cig, K).permute(0, 2, 3, 1).reshape(groups, Cig * K, Cog).contiguous()


def pack_convT(w: torch.Tensor, u: int) -> tuple[torch.Tensor, int]:
    """ConvTranspose1d weight [Ci, Co, K] (stride u) -> polyphase KM [u][Ci*T][Co], T = ceil(K/u).

    Phase r computes outputs t with (t + pad) % u == r as a stride-1 conv over x with taps
    tp in [0, T): x[q - (T-1) + tp] * W[ci][co][r + (T-1-tp)*u]  (zero where that tap >= K)."""
    Ci, Co, K = w.shape
    T = -(-K // u)
    out = torch.zeros(u, Ci, T, Co, dtype=w.dtype)
    for r in range(u):
        for tp in range(T):
            j = r + (T - 1 - tp) * u
            if j < K:
                out[r, :, tp, :] = w[:, :, j]
    return out.reshape(u, Ci * T, Co).contiguous(), T


# Split-bf16 engine switch (the f32-MFMA engine runs when off); RVC_AMD_X6=0 disables it.
X6 = os.environ.get("RVC_AMD_X6", "1") != "0"

# Arithmetic of the split-operand MFMA engine (f32 accumulation always):
#   "fp32"   f32-equivalent (the default; BASELINE configs 1-2, 4): "fp32x6" everywhere except the convs where
#            "f16x3" measured faster (conv_passes, rb_passes; F16_MIX; RVC_AMD_F16MIX=0 turns it off)
#   "fp32x6" 6 bf16 passes, f32-accurate products (~2^-22 relative per product)
#   "fp32sa" "fp32x6" with the 5 correction passes accumulated apart from hH (RMVPE, whose f0 is a per-frame
#            decision: the large sum is rounded once per 32 products, scripts/conv_prec.py)
#   "f16x3"  3 fp16 passes over power-of-2-scaled 22-bit operands (~2^-20 relative per product)
#   "bf16x3" 3 bf16 passes, 16-bit operand mantissas (~2^-16 relative per product)
#   "bf16"   1 pass, bf16 operands (BASELINE configs 3 and 5)
F16X3 = 16  # RVC_ARITH_F16X3
PASSES = {"fp32": 6, "fp32x6": 6, "fp32sa": 7, "f16x3": F16X3, "bf16x3": 3, "bf16": 1}
F16_MIX = os.environ.get("RVC_AMD_F16MIX", "1") != "0"
# with the producer's |max| (amax side channel), split-fp16 for every stride-1 1-D conv (RVC_AMD_AMAX_F16ALL=0: only
# where conv_passes picks it anyway; the cell then just replaces the per-tile pre-pass)
AMAX_F16ALL = os.environ.get("RVC_AMD_AMAX_F16ALL", "1") != "0"
AMAX_SHARDS = 64  # RVC_AMAX_SHARDS: u32 words per |max| cell
# round 6: the stride-2 convs with a producer's |max| (ContentVec's feature extractor) in split-fp16 too
# (RVC_AMD_AMAX_S2=0: 6-pass split-bf16 there, the round-5 form; rvc_model_common's conv_passes reads the same switch)
AMAX_S2 = os.environ.get("RVC_AMD_AMAX_S2", "1") != "0"


def conv_passes(K, Ci, stride=1, two_d=False, amax=False):
    """The pass set a conv launch runs at under the current precision (see PASSES): in "fp32", split-fp16
    where it measured faster than 6-pass split-bf16 (scripts/conv_bench.py, same box: k >= 7 up to 256
    input channels, and k = 3 at 64-128 channels; 6-pass at k = 3 over 256 or 32 channels) -- and every stride-1
    1-D conv whose input's |max| comes from its producer (``amax``: no per-tile pre-pass, which is what made the
    short-tap and wide convs slower in split-fp16)."""
    if _PRECISION == "fp32" and F16_MIX and not two_d and \
            ((stride == 1 and ((amax and AMAX_F16ALL) or (K >= 7 and Ci <= 256) or (K >= 3 and 64 <= Ci <= 128))) or
             (stride == 2 and amax and AMAX_F16ALL and AMAX_S2)):
        return F16X3
    return PASSES[_PRECISION]
_PRECISION = os.environ.get("RVC_AMD_PRECISION", "fp32")
if _PRECISION not in PASSES:
    raise ValueError(f"RVC_AMD_PRECISION must be one of {sorted(PASSES)}")


def get_precision() -> str:
    return _PRECISION


def set_precision(name: str) -> str:
    """Set the conv engine's arithmetic for subsequent launches; returns the previous setting."""
    global _PRECISION
    if name not in PASSES:
        raise ValueError(f"precision must be one of {sorted(PASSES)}, got {name!r}")
    prev, _PRECISION = _PRECISION, name
    return prev


class splitk_target:
    """Context manager: the conv engine's split-K target grid for the launches issued inside (tiles below which a
    conv's k range is split over blocks; 0 = never split, None = leave the current setting)."""

    def __init__(self, target):
        self.target = target

    def __enter__(self):
        if self.target is not None:
            self.prev = _lib.load().rvc_conv1d_set_splitk_target(int(self.target))
        return self

    def __exit__(self, *a):
        if self.target is not None:
            _lib.load().rvc_conv1d_set_splitk_target(self.prev)


class precision:
    """Context manager: ``with ops.precision("bf16"): ...``."""

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.prev = set_precision(self.name)
        return self

    def __exit__(self, *a):
        set_precision(self.prev)


class SplitImages:
    """The two operand images of one weight for the split-operand engine: ``bf`` (rvc_conv1d_pack_x6, the
    bf16 planes every bf16 pass count reads) and ``hf`` (rvc_conv1d_pack_f16, fp16 planes + row scales)."""

    def __init__(self, bf, hf):
        self.bf, self.hf = bf, hf

    def for_passes(self, passes):
        return self.hf if passes == F16X3 else self.bf

    def data_ptr(self, passes=None):
        return self.for_passes(PASSES[_PRECISION] if passes is None else passes).data_ptr()


def pack_x6(w_km: torch.Tensor, nphase: int, Ci: int, K: int, Co: int):
    """Device KM weights [nphase][Ci*K][Co] -> (SplitImages, nmf): the split-bf16 image
    (rvc_conv1d_pack_x6) and the split-fp16 image (rvc_conv1d_pack_f16) for the split-operand engine, or
    (None, 0) when the engine is off."""
    if not X6:
        return None, 0
    lib = _lib.load()
    imgs = []
    for size_fn, pack_fn in ((lib.rvc_conv1d_x6_bytes, lib.rvc_conv1d_pack_x6),
                             (lib.rvc_conv1d_f16_bytes, lib.rvc_conv1d_pack_f16)):
        nbytes = size_fn(nphase, Ci, K, Co)
        if nbytes <= 0:
            raise ValueError("pack_x6: bad shape")
        out = torch.empty(nbytes, dtype=torch.uint8, device=w_km.device)
        nmf = ctypes.c_int(0)
        check(pack_fn(_p(w_km), nphase, Ci, K, Co, ctypes.c_void_p(out.data_ptr()), ctypes.byref(nmf), _stream()),
              "conv1d_pack")
        imgs.append(out)
    return SplitImages(*imgs), nmf.value


class Conv:
    """A packed Conv1d (weight [Co, Ci/g, K], bias [Co]) resident on the device, with the split-operand images
    (pack_x6) the library's engine reads."""

    def __init__(self, w, b=None, groups=1, device="cuda"):
        self.Co, self.Cig, self.K = (int(s) for s in w.shape)
        self.groups = groups
        self.Ci = self.Cig * groups
        self.w = pack_km(w.float(), groups).to(device)
        self.b = b.float().to(device) if b is not None else None
        # the split-operand engine takes ungrouped convs with <= 64 taps (X6_K_MAX / x6_eligible in conv1d.hip;
        # CREPE's k=64 layers are the widest) and grouped ones with <= 128 (ContentVec's pos_conv), whose image holds
        # the groups as phases (ConvParams.gx6)
        if groups == 1 and self.K <= 64:
            self.wx, self.wx_nmf = pack_x6(self.w, 1, self.Ci, self.K, self.Co)
        elif groups > 1 and self.K <= 128:
            self.wx, self.wx_nmf = pack_x6(self.w, groups, self.Cig, self.K, self.Co // groups)
        else:
            self.wx, self.wx_nmf = None, 0

    def __call__(self, x, Lout=None, stride=1, pad=0, dil=1, **kw):
        return conv1d(x, self.w, self.Ci, self.Co, self.K, bias=self.b, stride=stride, pad=pad, dil=dil,
                      groups=self.groups, Lout=Lout, wx=self.wx, wx_nmf=self.wx_nmf, **kw)


class ConvT:
    """ConvTranspose1d(Ci, Co, K, stride u, padding p, output_padding 0) as u phase convs."""

    def __init__(self, w, b, u, pad, device="cuda"):
        self.Ci, self.Co, self.K = (int(s) for s in w.shape)
        self.u, self.pad = u, pad
        wp, self.T = pack_convT(w.float(), u)
        self.w = wp.to(device)
        self.b = b.float().to(device)
        self.wx, self.wx_nmf = pack_x6(self.w, u, self.Ci, self.T, self.Co)

    def out_len(self, Lin):
        return (Lin - 1) * self.u - 2 * self.pad + self.K

    def __call__(self, x, out=None, **kw):
        B, Ci, Lin = _shape3(x)
        Lout = self.out_len(Lin)
        ncols = (Lout - 1 + self.pad) // self.u + 1
        return conv1d(x, self.w, Ci, self.Co, self.T, bias=self.b, stride=1, pad=self.T - 1, dil=1, Lout=Lout,
                      ncols=ncols, nphase=self.u, ostride=self.u, ooffset=-self.pad, out=out,
                      flops=2.0 * B * Ci * self.Co * self.K * Lin, wx=self.wx, wx_nmf=self.wx_nmf, **kw)


class AmaxSlots:
    """n |max| cells (the conv engine's amax side channel, AMAX_SHARDS words each) for one pass of B batch elements,
    zeroed by one launch: ``s[k]`` is cell k -- B consecutive cells, one per batch element (element b's |max| at word
    b * AMAX_SHARDS: a clip's split-fp16 scale never depends on the other clips of its batch) -- handed to a producer
    as ``amax_out`` and to its consumers as ``amax_in``."""

    def __init__(self, n, device, B=1):
        self.B = B
        self.words = torch.zeros(n * B * AMAX_SHARDS, dtype=torch.int32, device=device)

    def __getitem__(self, k):
        w = self.B * AMAX_SHARDS
        return self.words[k * w:(k + 1) * w]


def amax_value(cell, b=0):
    """The |max| a cell holds for batch element b (the largest of its words, read back as f32)."""
    import numpy as np
    words = cell[b * AMAX_SHARDS:(b + 1) * AMAX_SHARDS].cpu().numpy().astype(np.int32)
    return float(words.view(np.float32).max())


LAST_CONV_FLOPS = 0.0
LAST_CONV_ENGINE = 0  # 0 = f32 MFMA engine, 1 = split-bf16 (x6) engine
LAST_CONV_PASSES = 0  # the split-operand launch's pass set (PASSES values; F16X3 = split-fp16), 0 = f32 engine
LAST_CONV_WS = 0  # its split-K workspace bytes (0 = not split)
_WS = {}
_WS_PRIVATE = None  # a workspace store owned by a captured graph (private_workspaces)


class private_workspaces:
    """``with ops.private_workspaces(store):`` -- split-K / split-KV / decode scratch comes from ``store``
    (a dict the caller keeps) instead of the shared per-stream pool.  A captured graph bakes the raw
    workspace pointers into its kernel nodes, so it must own them: buffers in a private store are never
    freed while the store lives (a grown buffer's predecessor is retired into the store, not released),
    and no eager launch or other graph draws from it (graph.ClipGraph)."""

    def __init__(self, store: dict):
        self.store = store

    def __enter__(self):
        global _WS_PRIVATE
        self.prev, _WS_PRIVATE = _WS_PRIVATE, self.store
        return self.store

    def __exit__(self, *a):
        global _WS_PRIVATE
        _WS_PRIVATE = self.prev


def _workspace(device, nbytes, kind="conv"):
    """Split-K / split-KV scratch per (device, stream), grown on demand: reuse is stream-ordered, and
    work running concurrently on another stream (VC's side stream) gets its own buffer."""
    key = f"{device}/{kind}/{torch.cuda.current_stream(device).stream_id}"
    pool = _WS if _WS_PRIVATE is None else _WS_PRIVATE
    buf = pool.get(key)
    if buf is None or buf.numel() * 4 < nbytes:
        if buf is not None and _WS_PRIVATE is not None:
            pool.setdefault("_retired", []).append(buf)  # a captured node may still point at it
        buf = torch.empty((nbytes + 3) // 4 + (1 << 20), dtype=torch.float32, device=device)
        pool[key] = buf
    return buf


def _room(t):
    """Elements addressable from t.data_ptr() to the end of its storage (views of batched buffers are
    strided: their numel understates what a kernel with batch strides may touch)."""
    return t.untyped_storage().nbytes() // t.element_size() - t.storage_offset()


def _shape3(x):
    if x.dim() == 2:
        return 1, x.shape[0], x.shape[1]
    return x.shape[0], x.shape[1], x.shape[2]


def conv1d(x, w, Ci, Co, K, *, bias=None, bias2=None, stride=1, pad=0, dil=1, groups=1, Lout=None, ncols=0,
           nphase=1, ostride=1, ooffset=0, out=None, res=None, in_act=ACT_NONE, in_slope=0.0, in_scale=1.0,
           out_act=ACT_NONE, out_slope=0.0, out_scale=1.0, accumulate=False, B=None, Lin=None, x_bstride=0,
           w_bstride=0, y_bstride=0, res_bstride=0, toff=None, wrap=0, flops=None, wx=None, wx_nmf=0,
           amax_in=None, amax_out=None, src=None):
    """y = conv(pre(x)) with fused epilogue.  x: [B][Ci][Lin] device f32 (t contiguous).

    ``amax_out`` / ``amax_in``: cells of the |max| side channel (``AmaxSlots``: AMAX_SHARDS words per batch element)
    -- the launch folds max |y| into ``amax_out`` (zeroed beforehand), and a split-fp16 launch takes its activation
    scale from ``amax_in`` (the producer's cell for x) instead of a per-tile pre-pass (include/rvc_amd.h).

    ``src`` = (conv, signal [B][N], stride, pad): the fused source conv -- every stored output also adds
    ``conv(signal)[m][t]`` of a 1-input-channel ``ops.Conv`` (the NSF generator's noise_convs, synthesizers.py:156),
    the same bits as that conv run separately with ``accumulate`` (rvc_conv1d_args.src_*).

    ``flops`` is the launch's ALGORITHMIC FLOP count for roofline accounting (recorded in
    LAST_CONV_FLOPS); the default is 2*B*Co*(Ci/g)*K*(valid outputs)."""
    global LAST_CONV_FLOPS, LAST_CONV_ENGINE, LAST_CONV_PASSES, LAST_CONV_WS
    if B is None:
        B, Cx, Lx = _shape3(x)
        if Lin is None:
            Lin = Lx
        if Cx != Ci:
            raise ValueError(f"conv1d: x has {Cx} channels, weight expects {Ci}")
        if not x.is_contiguous():
            raise ValueError("conv1d: x must be contiguous")
    if Lout is None:
        Lout = (Lin + 2 * pad - dil * (K - 1) - 1) // stride + 1
    if Lout <= 0:
        raise ValueError("conv1d: empty output")
    Cig = Ci // groups
    need_w = nphase * Cig * K * Co
    if w.numel() < need_w or (w_bstride and w.numel() < need_w + (B - 1) * w_bstride):
        raise ValueError("conv1d: packed weight too small")
    if out is None:
        out = torch.empty(B, Co, Lout, device=x.device, dtype=torch.float32) if B > 1 else \
            torch.empty(Co, Lout, device=x.device, dtype=torch.float32)
    elif _room(out) < (B - 1) * (y_bstride or Co * Lout) + Co * Lout:
        raise ValueError("conv1d: output buffer too small")
    if res is not None and _room(res) < (B - 1) * (res_bstride or Co * Lout) + Co * Lout:
        raise ValueError("conv1d: residual too small")
    if _room(x) < (B - 1) * (x_bstride or Ci * Lin) + Ci * Lin:
        raise ValueError("conv1d: input buffer too small")
    if bias is not None and bias.numel() < Co:
        raise ValueError("conv1d: bias too small")
    a = _lib.Conv1dArgs()
    a.x, a.w, a.bias, a.bias2, a.res, a.y = _p(x), _p(w), _p(bias), _p(bias2), _p(res), _p(out)
    a.B, a.Ci, a.Co, a.Lin, a.Lout, a.ncols = B, Ci, Co, Lin, Lout, ncols
    a.x_bstride, a.y_bstride, a.res_bstride, a.w_bstride = x_bstride, y_bstride, res_bstride, w_bstride
    a.K, a.stride, a.dil, a.pad, a.groups = K, stride, dil, pad, groups
    a.nphase, a.ostride, a.ooffset = nphase, ostride, ooffset
    a.in_act, a.out_act, a.accumulate = in_act, out_act, int(bool(accumulate))
    a.in_scale, a.in_slope, a.out_slope, a.out_scale = in_scale, in_slope, out_slope, out_scale
    if toff is not None:
        if len(toff) != K or K > 16:
            raise ValueError("conv1d: toff must have K <= 16 entries")
        a.ntoff = K
        for i, v in enumerate(toff):
            a.toff[i] = int(v)
    a.wrap = wrap
    a.amax_in, a.amax_out = _p(amax_in), _p(amax_out)
    for cell in (amax_in, amax_out):
        if cell is not None and cell.numel() < B * AMAX_SHARDS:
            raise ValueError(f"conv1d: a |max| cell needs {AMAX_SHARDS} words per batch element (B={B})")
    if src is not None:
        sconv, sig, s_stride, s_pad = src
        if sconv.Ci != 1 or sconv.groups != 1 or sconv.Co != Co:
            raise ValueError("conv1d: src needs a 1-input-channel conv with the output's channels")
        s_len = sig.shape[-1]
        if sig.dim() not in (1, 2) or (sig.dim() == 2 and sig.shape[0] != B) or not sig.is_contiguous() or \
                (sig.dim() == 1 and B != 1):
            raise ValueError("conv1d: src signal must be contiguous [B][N]")
        a.src_x, a.src_w, a.src_b = _p(sig), _p(sconv.w), _p(sconv.b)
        a.src_K, a.src_stride, a.src_pad, a.src_len, a.src_bstride = sconv.K, s_stride, s_pad, s_len, s_len
    if wx is not None:
        passes = conv_passes(K, Ci // groups, stride, toff is not None, amax_in is not None)
        a.wx, a.wx_nmf, a.wx_passes = ctypes.c_void_p(wx.data_ptr(passes)), wx_nmf, passes
    if flops is None:
        valid = (Lout // wrap - 2) * (wrap - 2) if wrap else (ncols or Lout) * nphase
        flops = 2.0 * B * Co * Cig * K * min(valid, Lout)
    LAST_CONV_FLOPS = flops
    lib = _lib.load()
    need = lib.rvc_conv1d_workspace_bytes(ctypes.byref(a))
    if need < 0:
        raise RuntimeError(f"rvc_amd: conv1d plan failed: {lib.rvc_last_error().decode()}")
    ws = _workspace(out.device, need) if need else None
    LAST_CONV_WS = need
    LAST_CONV_ENGINE = lib.rvc_conv1d_engine(ctypes.byref(a))
    LAST_CONV_PASSES = a.wx_passes if LAST_CONV_ENGINE == 1 else 0
    check(lib.rvc_conv1d(ctypes.byref(a), _p(ws), need, _stream()), "conv1d")
    return out


# Fused ResBlock pairs for the 32/64-channel generator stages (RVC_AMD_FUSED_RB=0: two conv launches each)
FUSED_RB = os.environ.get("RVC_AMD_FUSED_RB", "1") != "0"
RB_PASSES = (6, 3, 1, F16X3)  # pass sets the fused kernel takes


# the fused pair's smallest split-fp16 kernel size (RVC_AMD_RB_F16_KMIN, A/B switch): 3 since round 5 (C = 64 K = 3
# pairs 371 -> 327 us, C = 32 250 -> 231, clip stream +0.6 %; scripts/gpu_r5_rbk3.sh), 7 before
RB_F16_KMIN = int(os.environ.get("RVC_AMD_RB_F16_KMIN", "3"))


def rb_passes(K):
    """The fused ResBlock pair's pass set under the current precision: "fp32" mixes in split-fp16 for
    k >= RB_F16_KMIN (round 2: 7-8 % faster at k >= 7 and slower at k = 3; round 5: faster at k = 3 too)."""
    if _PRECISION == "fp32" and F16_MIX and K >= RB_F16_KMIN:
        return F16X3
    return PASSES[_PRECISION]


# the 128-channel fused pair (round 4; <= 2 split planes fit LDS: pass sets 3, 1, F16X3): correct (bit-identical to
# two launches, tests/test_gpu_resblock.py) but measured slower in the clip stream (893 vs 920 xRT), so only on
# request: RVC_AMD_FUSED_RB128=1
FUSED_RB128 = os.environ.get("RVC_AMD_FUSED_RB128", "0") != "0"


def resblock_fusable(c1: "Conv", c2: "Conv", dil: int) -> bool:
    passes = rb_passes(c1.K)
    chans = c1.Co in (32, 64) or (c1.Co == 128 and FUSED_RB128 and passes in (3, 1, F16X3))
    return (FUSED_RB and passes in RB_PASSES and c1.wx is not None and c2.wx is not None
            and c1.Ci == c1.Co == c2.Ci == c2.Co
            and chans and c1.K == c2.K and c1.K % 2 == 1 and c1.K <= 15 and (c1.K - 1) * dil <= 64)


def resblock_pair(x, y, c1: "Conv", c2: "Conv", dil: int, slope: float, accumulate: bool = False):
    """y (+)= x + c2(lrelu(c1(lrelu(x), dil)))  (residuals.py:22-44, one pair) in one launch; x [C][L] or
    [B][C][L] (B clips, each bit-identical to its own call)."""
    B, C, L = _shape3(x)
    if y.shape != x.shape or not x.is_contiguous() or not y.is_contiguous() or x.data_ptr() == y.data_ptr():
        raise ValueError("resblock_pair: x, y must be distinct contiguous [(B)][C][L] buffers")
    a = _lib.ResblockArgs()
    a.x, a.y = _p(x), _p(y)
    passes = rb_passes(c1.K)
    a.w1x, a.w2x = ctypes.c_void_p(c1.wx.data_ptr(passes)), ctypes.c_void_p(c2.wx.data_ptr(passes))
    a.b1, a.b2 = _p(c1.b), _p(c2.b)
    a.C, a.L, a.K, a.dil = C, L, c1.K, dil
    a.B = B
    a.nmf1, a.nmf2 = c1.wx_nmf, c2.wx_nmf
    a.passes, a.accumulate, a.slope = passes, int(bool(accumulate)), slope
    check(_lib.load().rvc_resblock_pair(ctypes.byref(a), _stream()), "resblock_pair")
    return y


def attention(q, k, v, o, *, B, H, D, T, ldc, q_hs, k_hs, v_hs, o_hs, scale, q_bs=0, k_bs=0, v_bs=0, o_bs=0,
              rk=None, ev=None, ml=None, W=0, amax_out=None, amax_in=None):
    """Flash attention (rvc_attention_ex); ``amax_out``: a |max| cell (``AmaxSlots``) that receives max |o|;
    ``amax_in``: the cell holding max |q|, |k|, |v| (the QKV projection's) -- both products then run in split-fp16
    on the fp16 matrix cores (round 6; ``rvc_attention_set_f16`` / RVC_ATTN_F16=0 keep the f32 kernel)."""
    a = _lib.AttnArgs()
    a.q, a.k, a.v, a.o, a.rk, a.ev, a.ml = _p(q), _p(k), _p(v), _p(o), _p(rk), _p(ev), _p(ml)
    a.B, a.H, a.D, a.T, a.ldc = B, H, D, T, ldc
    a.q_hs, a.k_hs, a.v_hs, a.o_hs = q_hs, k_hs, v_hs, o_hs
    a.q_bs, a.k_bs, a.v_bs, a.o_bs = q_bs, k_bs, v_bs, o_bs
    a.W, a.scale = W, scale
    lib = _lib.load()
    need = lib.rvc_attention_workspace_bytes(ctypes.byref(a))
    if need < 0:
        raise ValueError(f"attention: unsupported shape H={H} D={D} T={T}")
    ws = _workspace(o.device, need, "attn") if need else None
    for cell in (amax_in, amax_out):
        if cell is not None and cell.numel() < B * AMAX_SHARDS:
            raise ValueError("attention: a |max| cell needs AMAX_SHARDS words per batch element")
    check(lib.rvc_attention_ex(ctypes.byref(a), _p(amax_in), _p(amax_out), _p(ws), need, _stream()), "attention")
    return o


def textenc_embed(lin, emb, pitch, out, B, C, T, scale, slope, amax_out=None):
    """``amax_out``: a |max| cell (``AmaxSlots``) that receives max |out| per batch element."""
    if amax_out is not None and amax_out.numel() < B * AMAX_SHARDS:
        raise ValueError("textenc_embed: amax_out needs a cell per batch element")
    check(_lib.load().rvc_textenc_embed_amax(_p(lin), _p(emb), _p(pitch), _p(out), B, C, T, scale, slope,
                                             _p(amax_out), _stream()), "textenc_embed")
    return out


def layernorm_cf(x, res, gamma, beta, out, B, C, T, eps=1e-5, amax_out=None):
    """LayerNorm over channels of x (+ res); ``amax_out``: a |max| cell that receives max |out|."""
    if x.numel() < B * C * T or out.numel() < B * C * T or gamma.numel() < C:
        raise ValueError("layernorm_cf: size mismatch")
    if amax_out is not None:
        check(_lib.load().rvc_layernorm_cf_amax(_p(x), _p(res), _p(gamma), _p(beta), _p(out), B, C, T, eps,
                                                _p(amax_out), _stream()), "layernorm_cf")
    else:
        check(_lib.load().rvc_layernorm_cf(_p(x), _p(res), _p(gamma), _p(beta), _p(out), B, C, T, eps, _stream()),
              "layernorm_cf")
    return out


def chnorm_gelu(x, gamma, beta, out, B, C, L, eps=1e-5, gelu=True):
    if x.numel() < B * C * L or out.numel() < B * C * L:
        raise ValueError("chnorm_gelu: size mismatch")
    check(_lib.load().rvc_chnorm_gelu(_p(x), _p(gamma), _p(beta), _p(out), B, C, L, eps, int(gelu), _stream()),
          "chnorm_gelu")
    return out


def fe0_gn_gelu(wav, w_km, gamma, beta, B, N, C, K, stride, eps=1e-5, gelu=True, x_bstride=0, amax_out=None):
    """ContentVec's first layer fused: conv(1 -> C, k K, stride) of wav [B][N] + GroupNorm(C, C) + affine + GELU
    -> [B][C][T] (rvc_fe0_gn_gelu; w_km: the K-major packed conv weight [K][C], ops.Conv.w); ``amax_out``: a |max|
    cell (``AmaxSlots``) that receives max |out| per batch element (rvc_fe0_gn_gelu_amax)."""
    lib = _lib.load()
    T = (N - K) // stride + 1
    out = torch.empty(B, C, T, device=wav.device) if B > 1 else torch.empty(C, T, device=wav.device)
    need = lib.rvc_fe0_ws_bytes(B, C, T)
    ws = _workspace(wav.device, need, kind="fe0")
    if amax_out is not None and amax_out.numel() < B * AMAX_SHARDS:
        raise ValueError("fe0_gn_gelu: amax_out needs a cell per batch element")
    check(lib.rvc_fe0_gn_gelu_amax(_p(wav), B, N, x_bstride, _p(w_km), C, K, stride, _p(gamma), _p(beta), _p(out),
                                   eps, int(gelu), _p(amax_out), _p(ws), need, _stream()), "fe0_gn_gelu")
    return out


def prior_sample(stats, noise, zp, B, C, T, nscale=0.66666):
    check(_lib.load().rvc_prior_sample(_p(stats), _p(noise), _p(zp), B, C, T, nscale, _stream()), "prior_sample")
    return zp


def gate(a, out, B, H, T):
    check(_lib.load().rvc_gate(_p(a), _p(out), B, H, T, _stream()), "gate")
    return out


def flip_channels(x, out, B, C, T):
    check(_lib.load().rvc_flip_channels(_p(x), _p(out), B, C, T, _stream()), "flip")
    return out


def transpose(x, out, B, R, C):
    check(_lib.load().rvc_transpose(_p(x), _p(out), B, R, C, _stream()), "transpose")
    return out


# Device-resident seed added to every Philox draw while set (graph.ClipGraph: replays draw fresh noise).
_DEV_SEED = None


class device_seed:
    """``with ops.device_seed(t):`` -- t: device int64 [1]; draws use seed + t[0], read at run time."""

    def __init__(self, t):
        self.t = t

    def __enter__(self):
        global _DEV_SEED
        self.prev, _DEV_SEED = _DEV_SEED, self.t
        return self

    def __exit__(self, *a):
        global _DEV_SEED
        _DEV_SEED = self.prev


def graph_mode() -> bool:
    """True while a device seed is set, i.e. while ClipGraph warms up or captures."""
    return _DEV_SEED is not None


def randn(out, seed, offset=0):
    add = _p(_DEV_SEED) if _DEV_SEED is not None else None
    check(_lib.load().rvc_randn_ex(_p(out), out.numel(), seed, offset, add, _stream()), "randn")
    return out


def rand_triang(out, lo, hi, seed, offset=0):
    """Symmetric triangular draws on [lo, hi] (Philox counter stream; device seed added when set)."""
    add = _p(_DEV_SEED) if _DEV_SEED is not None else None
    check(_lib.load().rvc_rand_triang(_p(out), out.numel(), lo, hi, seed, offset, add, _stream()), "rand_triang")
    return out


def sine_source(f0, noise, har, work, B, T, upp, sr, lin_w, lin_b):
    if f0.numel() < B * T or noise.numel() < B * T * upp or har.numel() < B * T * upp or work.numel() < B * T:
        raise ValueError("sine_source: size mismatch")
    check(_lib.load().rvc_sine_source(_p(f0), _p(noise), _p(har), _p(work), B, T, upp, sr, lin_w, lin_b, _stream()),
          "sine_source")
    return har


def stft_frames(x, win, out, N, F, nfft, hop):
    if x.numel() < N or win.numel() < nfft or out.numel() < nfft * F:
        raise ValueError("stft_frames: size mismatch")
    check(_lib.load().rvc_stft_frames(_p(x), _p(win), _p(out), N, F, nfft, hop, _stream()), "stft_frames")
    return out


def stft_mag(x, win, mag, N, F, nfft, hop):
    """|STFT| in f64, rounded once: x [N] or [B][N] -> mag [nfft/2+1][F] or [B][nfft/2+1][F]."""
    B = x.shape[0] if x.dim() == 2 else 1
    K = nfft // 2 + 1
    if (x.shape[-1] < N or win.numel() < nfft or mag.numel() < B * K * F or mag.shape[-1] != F
            or (B > 1 and (mag.dim() != 3 or mag.shape[0] != B))):
        raise ValueError("stft_mag: size mismatch")
    if x.stride(-1) != 1 or mag.stride(-1) != 1:
        raise ValueError("stft_mag: x / mag rows must be contiguous")
    xs = x.stride(0) if B > 1 else 0
    ms = mag.stride(0) if B > 1 else 0
    check(_lib.load().rvc_stft_mag(_p(x), _p(win), _p(mag), B, N, F, nfft, hop, xs, ms, _stream()), "stft_mag")
    return mag


def spec_mag(spec, mag, K, F):
    if spec.numel() < 2 * K * F or mag.numel() < K * F:
        raise ValueError("spec_mag: size mismatch")
    check(_lib.load().rvc_spec_mag(_p(spec), _p(mag), K, F, _stream()), "spec_mag")
    return mag


def mel_image(mel, img, M, F, Tp, scale, shift):
    if mel.numel() < M * F or img.numel() < (Tp + 2) * (M + 2):
        raise ValueError("mel_image: size mismatch")
    check(_lib.load().rvc_mel_image(_p(mel), _p(img), M, F, Tp, scale, shift, _stream()), "mel_image")
    return img


def avgpool2(x, out, C, H, W):
    if x.numel() < C * (H + 2) * (W + 2) or out.numel() < C * (H // 2 + 2) * (W // 2 + 2):
        raise ValueError("avgpool2: size mismatch")
    check(_lib.load().rvc_avgpool2(_p(x), _p(out), C, H, W, _stream()), "avgpool2")
    return out


def interleave4(phases, out, C, H, W):
    if phases.numel() < 4 * C * (H + 2) * (W + 2) or out.numel() < C * (2 * H + 2) * (2 * W + 2):
        raise ValueError("interleave4: size mismatch")
    check(_lib.load().rvc_interleave4(_p(phases), _p(out), C, H, W, _stream()), "interleave4")
    return out


def img_to_seq(img, x, C, H, W):
    if img.numel() < C * (H + 2) * (W + 2) or x.numel() < C * W * H:
        raise ValueError("img_to_seq: size mismatch")
    check(_lib.load().rvc_img_to_seq(_p(img), _p(x), C, H, W, _stream()), "img_to_seq")
    return x


def bigru(gi, whh, bhh, y, gran, err, T):
    if gi.numel() < 2 * 768 * T or whh.numel() < 2 * 768 * 256 or y.numel() < 512 * T or gran.numel() < 1024:
        raise ValueError("bigru: size mismatch")
    check(_lib.load().rvc_bigru(_p(gi), _p(whh), _p(bhh), _p(y), _p(gran), _p(err), T, _stream()), "bigru")
    return y


GRU_B_MAX = 16  # sequences per bigru launch (rvc_bigru_batched); gran scratch is 1024 int64 per sequence


def bigru_batched(gi, whh, bhh, y, gran, err, B, T):
    """B independent BiGRU recurrences: gi [B][1536][T], y [B][512][T] (batch strides from the tensors)."""
    if gi.dim() != 3 or y.dim() != 3 or gi.shape[0] < B or y.shape[0] < B or gi.shape[1] != 1536 or y.shape[1] != 512:
        raise ValueError("bigru_batched: gi [B][1536][T], y [B][512][T] expected")
    if gi.shape[2] < T or y.shape[2] < T or gran.numel() < 1024 * min(B, GRU_B_MAX) or whh.numel() < 2 * 768 * 256:
        raise ValueError("bigru_batched: size mismatch")
    check(_lib.load().rvc_bigru_batched(_p(gi), gi.stride(0), _p(whh), _p(bhh), _p(y), y.stride(0), _p(gran), _p(err),
                                        B, T, _stream()), "bigru_batched")
    return y


# ------------------------------------------------------------------ f64 RMVPE (rmvpe64.hip)
def _pd(t):
    if t is None:
        return None
    if not t.is_cuda or t.dtype != torch.float64:
        raise TypeError(f"rvc_amd: expected a CUDA f64 tensor, got {t.dtype} on {t.device}")
    return ctypes.c_void_p(t.data_ptr())


class Conv64:
    """A Conv weight [Co, Ci, K] (and bias [Co]) kept in f64 KM layout for ``conv64``."""

    def __init__(self, w, b=None, device="cuda"):
        self.Co, self.Ci, self.K = (int(s) for s in w.shape)
        self.w = pack_km(w.double()).to(device)
        self.b = b.double().to(device) if b is not None else None

    def __call__(self, x, Lout=None, **kw):
        return conv64(x, self.w, self.Ci, self.Co, self.K, bias=self.b, Lout=Lout, **kw)


def conv64(x, w, Ci, Co, K, *, bias=None, pad=0, Lout=None, out=None, res=None, out_act=ACT_NONE, out_slope=0.0,
           B=None, Lin=None, x_bstride=0, y_bstride=0, res_bstride=0, toff=None, wrap=0, out_f32=False, plan=False):
    """The f64 conv (rvc_conv64): x [B][Ci][Lin] f64, y f64 (or f32 when ``out_f32``), stride 1, K taps at
    ``toff`` (or 0..K-1), 2-D border masking with ``wrap``; see include/rvc_amd.h.  ``plan=True`` launches
    nothing and returns the planner's choice (rvc_conv64_plan): (tile, split-K, compact, blocks)."""
    if B is None:
        B, Cx, Lx = _shape3(x)
        if Lin is None:
            Lin = Lx
        if Cx != Ci:
            raise ValueError(f"conv64: x has {Cx} channels, weight expects {Ci}")
        if not x.is_contiguous():
            raise ValueError("conv64: x must be contiguous")
    if Lout is None:
        Lout = Lin + 2 * pad - (K - 1)
    if Lout <= 0:
        raise ValueError("conv64: empty output")
    if w.numel() < Ci * K * Co or w.dtype != torch.float64:
        raise ValueError("conv64: f64 KM weight [Ci*K][Co] expected")
    ydt = torch.float32 if out_f32 else torch.float64
    if out is None:
        out = torch.empty(*((B,) if B > 1 else ()), Co, Lout, device=x.device, dtype=ydt)
    elif out.dtype != ydt or _room(out) < (B - 1) * (y_bstride or Co * Lout) + Co * Lout:
        raise ValueError("conv64: output buffer too small or of the wrong dtype")
    if res is not None and _room(res) < (B - 1) * (res_bstride or Co * Lout) + Co * Lout:
        raise ValueError("conv64: residual too small")
    if _room(x) < (B - 1) * (x_bstride or Ci * Lin) + Ci * Lin:
        raise ValueError("conv64: input buffer too small")
    if bias is not None and bias.numel() < Co:
        raise ValueError("conv64: bias too small")
    a = _lib.Conv64Args()
    a.x, a.w, a.bias, a.res = _pd(x), _pd(w), _pd(bias), _pd(res)
    a.y = _p(out) if out_f32 else _pd(out)
    a.B, a.Ci, a.Co, a.Lin, a.Lout = B, Ci, Co, Lin, Lout
    a.x_bstride, a.y_bstride, a.res_bstride = x_bstride, y_bstride, res_bstride
    a.K, a.pad, a.out_act, a.y_f32, a.out_slope = K, pad, out_act, int(bool(out_f32)), out_slope
    if toff is not None:
        if len(toff) != K or K > 16:
            raise ValueError("conv64: toff must have K <= 16 entries")
        a.ntoff = K
        for i, v in enumerate(toff):
            a.toff[i] = int(v)
    a.wrap = wrap
    lib = _lib.load()
    if plan:
        res4 = (ctypes.c_int * 4)()
        check(lib.rvc_conv64_plan(ctypes.byref(a), res4), "conv64_plan")
        return tuple(res4)
    need = lib.rvc_conv64_workspace_bytes(ctypes.byref(a))
    if need < 0:
        raise RuntimeError(f"rvc_amd: conv64 plan failed: {lib.rvc_last_error().decode()}")
    ws = _workspace(out.device, need, "c64") if need else None
    check(lib.rvc_conv64(ctypes.byref(a), _p(ws), need, _stream()), "conv64")
    return out


def wino64_use(Ci, Co, H=0, W=0):
    """Whether the f64 RMVPE takes the Winograd F(4x4, 3x3) form for a Ci -> Co 3x3 conv on an H x W image
    (rvc_wino64_use; H = W = 0: the channel rule alone, i.e. whether to prepare the transformed weights)."""
    return bool(_lib.load().rvc_wino64_use(Ci, Co, H, W))


def wino64_weights(w_km, Ci, Co):
    """KM f64 3x3 weights [Ci*9][Co] -> the 36 Winograd weight matrices [36][Ci][Co] (rvc_wino64_weights)."""
    v = torch.empty(36, Ci, Co, dtype=torch.float64, device=w_km.device)
    check(_lib.load().rvc_wino64_weights(_pd(w_km), _pd(v), Ci, Co, _stream()), "wino64_weights")
    return v


def wino64(x, v, Ci, Co, H, W, *, bias=None, res=None, out=None, out_act=ACT_NONE, B=1, x_bstride=0, y_bstride=0,
           res_bstride=0, out_f32=False):
    """The f64 Winograd F(4x4, 3x3) conv (rvc_wino64_conv) on bordered [Ci][H+2][W+2] images (or B of them with
    batch strides): y = act(conv3x3(x) + bias) (+ res), border cells 0."""
    L = (H + 2) * (W + 2)
    ydt = torch.float32 if out_f32 else torch.float64
    if out is None:
        out = torch.empty(*((B,) if B > 1 else ()), Co, H + 2, W + 2, device=x.device, dtype=ydt)
    elif out.dtype != ydt or _room(out) < (B - 1) * (y_bstride or Co * L) + Co * L:
        raise ValueError("wino64: output buffer too small or of the wrong dtype")
    if _room(x) < (B - 1) * (x_bstride or Ci * L) + Ci * L or x.dtype != torch.float64:
        raise ValueError("wino64: f64 input of [B][Ci][H+2][W+2] expected")
    if res is not None and _room(res) < (B - 1) * (res_bstride or Co * L) + Co * L:
        raise ValueError("wino64: residual too small")
    if v.numel() < 36 * Ci * Co or v.dtype != torch.float64:
        raise ValueError("wino64: f64 weights [36][Ci][Co] expected")
    a = _lib.Wino64Args()
    a.x, a.v, a.bias, a.res = _pd(x), _pd(v), _pd(bias), _pd(res)
    a.y = _p(out) if out_f32 else _pd(out)
    a.B, a.Ci, a.Co, a.H, a.W = B, Ci, Co, H, W
    a.x_bstride, a.y_bstride, a.res_bstride = x_bstride, y_bstride, res_bstride
    a.out_act, a.y_f32 = out_act, int(bool(out_f32))
    lib = _lib.load()
    need = lib.rvc_wino64_workspace_bytes(ctypes.byref(a))
    if need < 0:
        raise RuntimeError(f"rvc_amd: wino64 plan failed: {lib.rvc_last_error().decode()}")
    ws = _workspace(out.device, need, "w64")
    check(lib.rvc_wino64_conv(ctypes.byref(a), _p(ws), need, _stream()), "wino64")
    return out


def conv64_set_plan(tile=-1, ksplit=-1, compact=-1):
    """Force the f64 conv planner's choice (rvc_conv64_set_plan; -1 = the planner's): sweeps and tests."""
    check(_lib.load().rvc_conv64_set_plan(tile, ksplit, compact), "conv64_set_plan")


def _bs(t, nd):
    """Batch stride of a [B][...] view (0 for an unbatched tensor of ``nd`` dims)."""
    return t.stride(0) if t.dim() > nd else 0


def stft_mag64(x, win, mag, N, F, nfft, hop):
    """|STFT| in f64 (unrounded): x [N] or [B][N] f32 -> mag f64 [nfft/2+1][F] or [B][nfft/2+1][F]."""
    B = x.shape[0] if x.dim() == 2 else 1
    K = nfft // 2 + 1
    if (x.shape[-1] < N or win.numel() < nfft or mag.numel() < B * K * F or mag.shape[-1] != F
            or (B > 1 and (mag.dim() != 3 or mag.shape[0] != B))):
        raise ValueError("stft_mag64: size mismatch")
    if x.stride(-1) != 1 or mag.stride(-1) != 1:
        raise ValueError("stft_mag64: x / mag rows must be contiguous")
    check(_lib.load().rvc_stft_mag64(_p(x), _p(win), _pd(mag), B, N, F, nfft, hop, x.stride(0) if B > 1 else 0,
                                     mag.stride(0) if B > 1 else 0, _stream()), "stft_mag64")
    return mag


def mel_image64(mel, img, M, F, Tp, scale, shift):
    """mel [(B)][M][F] f64 -> interior of bordered images [(B)][1][Tp+2][M+2] f64 (reflect-padded frames)."""
    B = mel.shape[0] if mel.dim() == 3 else 1
    if mel.numel() < B * M * F or img.numel() < B * (Tp + 2) * (M + 2):
        raise ValueError("mel_image64: size mismatch")
    check(_lib.load().rvc_mel_image64(_pd(mel), _pd(img), B, M, F, Tp, scale, shift, _bs(mel, 2), _bs(img, 3),
                                      _stream()), "mel_image64")
    return img


def avgpool2_64(x, out, C, H, W):
    B = x.shape[0] if x.dim() == 4 else 1
    if _room(x) < B * C * (H + 2) * (W + 2) or _room(out) < B * C * (H // 2 + 2) * (W // 2 + 2):
        raise ValueError("avgpool2_64: size mismatch")
    check(_lib.load().rvc_avgpool2_64(_pd(x), _pd(out), B, C, H, W, _bs(x, 3), _bs(out, 3), _stream()), "avgpool2_64")
    return out


def interleave4_64(phases, out, C, H, W):
    """phases [(B)][4][C][H+2][W+2] -> the first C channels of bordered out [(B)][*][2H+2][2W+2]."""
    B = phases.shape[0] if phases.dim() == 5 else 1
    if _room(phases) < B * 4 * C * (H + 2) * (W + 2) or _room(out) < B * C * (2 * H + 2) * (2 * W + 2):
        raise ValueError("interleave4_64: size mismatch")
    check(_lib.load().rvc_interleave4_64(_pd(phases), _pd(out), B, C, H, W, _bs(phases, 4), _bs(out, 3), _stream()),
          "interleave4_64")
    return out


def img_to_seq64(img, x, C, H, W):
    B = img.shape[0] if img.dim() == 4 else 1
    if _room(img) < B * C * (H + 2) * (W + 2) or _room(x) < B * C * W * H:
        raise ValueError("img_to_seq64: size mismatch")
    check(_lib.load().rvc_img_to_seq64(_pd(img), _pd(x), B, C, H, W, _bs(img, 3), _bs(x, 2), _stream()),
          "img_to_seq64")
    return x


GRU64_GRAN = 16384 // 8  # int64 words of bigru64 hand-off scratch per sequence (RVC_BIGRU64_GRAN_BYTES)


def bigru64_batched(gi, whh, bhh, y, gran, err, B, T):
    """B f64 BiGRU recurrences: gi [(B)][1536][T], y [(B)][512][T] f64."""
    if gi.shape[-2] != 1536 or y.shape[-2] != 512 or gi.shape[-1] < T or y.shape[-1] < T:
        raise ValueError("bigru64: gi [(B)][1536][T], y [(B)][512][T] expected")
    if (gi.dim() == 3 and gi.shape[0] < B) or (y.dim() == 3 and y.shape[0] < B) or (B > 1 and gi.dim() != 3):
        raise ValueError("bigru64: batch mismatch")
    if gran.numel() < GRU64_GRAN * min(B, GRU_B_MAX) or whh.numel() < 2 * 768 * 256 or whh.dtype != torch.float64:
        raise ValueError("bigru64: size mismatch")
    check(_lib.load().rvc_bigru64_batched(_pd(gi), _bs(gi, 2), _pd(whh), _pd(bhh), _pd(y), _bs(y, 2), _p(gran), _p(err),
                                          B, T, _stream()), "bigru64")
    return y


class F0Post:
    """The optional steps of VC.get_f0 between the raw f0 and the quantiser (convert.py:311-318):
    autotune strength (None = off) and the f0-file override ``rep`` (f64 values for frames
    [rep_off, rep_off + len(rep)))."""

    def __init__(self, autotune_strength=None, rep=None, rep_off=0, device=None):
        self.autotune_strength = autotune_strength
        self.rep = None
        self.rep_off = int(rep_off)
        if rep is not None and len(rep) > 0:
            import numpy as np
            self.rep = torch.from_numpy(np.ascontiguousarray(rep, dtype=np.float64)).to(device)

    def struct(self, F):
        """ctypes rvc_f0_post for an f0 track of F frames (the override is clipped to it)."""
        s = _lib.F0Post()
        if self.autotune_strength is not None:
            s.autotune, s.strength = 1, float(self.autotune_strength)
        if self.rep is not None and self.rep_off < F:
            s.rep = ctypes.c_void_p(self.rep.data_ptr())
            s.rep_off, s.rep_len = self.rep_off, min(self.rep.numel(), F - self.rep_off)
        return s


def _post_ref(post, F):
    return ctypes.byref(post.struct(F)) if post is not None else None


def rmvpe_decode(sal, ld, F, thred, shift, f0, coarse, pitchf, post=None):
    if sal.numel() < 360 * ld or coarse.numel() < F or pitchf.numel() < F or (f0 is not None and f0.numel() < F):
        raise ValueError("rmvpe_decode: size mismatch")
    f0p = ctypes.c_void_p(f0.data_ptr()) if f0 is not None else None
    check(_lib.load().rvc_rmvpe_decode(_p(sal), ld, F, thred, shift, _post_ref(post, F), f0p, _p(coarse), _p(pitchf),
                                       _stream()), "rmvpe_decode")


class FiltFilt:
    """scipy.signal.filtfilt(b, a, .) + reflect padding on the device (filtfilt.hip); zi = lfilter_zi(b, a)
    is computed once on the host like the filter design itself."""

    def __init__(self, b, a):
        from scipy import signal
        import numpy as np
        self.b = np.ascontiguousarray(b, dtype=np.float64)
        self.a = np.ascontiguousarray(a, dtype=np.float64)
        if self.b.size != 6 or self.a.size != 6 or self.a[0] != 1.0:
            raise ValueError("FiltFilt: 5th-order filter with a[0] == 1 expected")
        self.zi = np.ascontiguousarray(signal.lfilter_zi(self.b, self.a), dtype=np.float64)

    def __call__(self, x, tpad, want_f64=False):
        """x: device f32 [N] -> (reflect-padded filtered f32 [N + 2 tpad], f64 copy or None)."""
        N = x.numel()
        nbytes = _lib.load().rvc_filtfilt_work_bytes(N)
        if nbytes < 0:
            raise ValueError(f"filtfilt: bad length {N}")
        work = torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=x.device)
        out = torch.empty(N + 2 * tpad, device=x.device)
        out64 = torch.empty(N + 2 * tpad, dtype=torch.float64, device=x.device) if want_f64 else None
        h = lambda arr: ctypes.c_void_p(arr.ctypes.data)  # noqa: E731
        check(_lib.load().rvc_filtfilt_pad(_p(x), N, h(self.b), h(self.a), h(self.zi), tpad,
                                           ctypes.c_void_p(work.data_ptr()), _p(out),
                                           ctypes.c_void_p(out64.data_ptr()) if want_f64 else None, _stream()),
              "filtfilt_pad")
        return out, out64


def quiet_points(x64, window, t_center, t_query, t_max):
    """VC.pipeline's quiet-point segmentation (convert.py:404-412) on the device: the filtered f64 signal
    x64 [n] (unpadded) -> host list of opt_ts (one small device->host copy; the segment plan needs it)."""
    lib = _lib.load()
    n = x64.numel()
    cnt = lib.rvc_quiet_points_count(n, window, t_center, t_max)
    if cnt < 0:
        raise ValueError("quiet_points: bad arguments")
    if cnt == 0:
        return []
    if x64.dtype != torch.float64 or not x64.is_cuda or not x64.is_contiguous():
        raise TypeError("quiet_points: a contiguous CUDA f64 signal")
    need = lib.rvc_quiet_points_ws_bytes(n, window, t_center, t_query, t_max)
    ws = _workspace(x64.device, need, "quiet")
    out = torch.empty(cnt, dtype=torch.int64, device=x64.device)
    check(lib.rvc_quiet_points(ctypes.c_void_p(x64.data_ptr()), n, window, t_center, t_query, t_max, _p(ws), need,
                               _p(out), _stream()), "quiet_points")
    return out.cpu().tolist()


IVF_FAISS, IVF_EXACT = 0, 1  # RVC_IVF_FAISS (faiss's own f32 arithmetic, the default) / RVC_IVF_EXACT (f64)


def ivf_search(q, nq, d, cs, qs, centT, nlist, nprobe, list_off, codes, ids, k, D, I, probes, arithmetic=IVF_FAISS):
    """FAISS IVF-Flat search (ivf.hip): see include/rvc_amd.h."""
    if D.numel() < nq * k or I.numel() < nq * k or probes.numel() < nq * nprobe or centT.numel() < d * nlist:
        raise ValueError("ivf_search: output / index buffers too small")
    if _room(q) < (d - 1) * cs + (nq - 1) * qs + 1:
        raise ValueError("ivf_search: query buffer too small")
    lib = _lib.load()
    need = lib.rvc_ivf_coarse_ws_bytes(nq, nlist)
    ws = _workspace(q.device, need, "ivf")
    check(lib.rvc_ivf_search_ex(_p(q), nq, d, cs, qs, _p(centT), nlist, nprobe, _p(list_off), _p(codes), _p(ids), k,
                                _p(ws), need, _p(probes), _p(D), _p(I), arithmetic, _stream()), "ivf_search")


def ivf_blend(feats, nq, d, fcs, fqs, D, I, k, big, ntotal, index_rate, out, ocs, oqs):
    if big.numel() < ntotal * d or D.numel() < nq * k or I.numel() < nq * k:
        raise ValueError("ivf_blend: buffers too small")
    check(_lib.load().rvc_ivf_blend(_p(feats), nq, d, fcs, fqs, _p(D), _p(I), k, _p(big), ntotal, float(index_rate),
                                    _p(out), ocs, oqs, _stream()), "ivf_blend")


def phone_upsample(feats, feats0, pitchf, out, C, Tf, T, protect):
    if feats.numel() < C * Tf or out.numel() < C * T or T > 2 * Tf or (pitchf is not None and pitchf.numel() < T):
        raise ValueError("phone_upsample: size mismatch")
    check(_lib.load().rvc_phone_upsample(_p(feats), _p(feats0), _p(pitchf), _p(out), C, Tf, T, protect, _stream()),
          "phone_upsample")
    return out


def peak_normalize(x, ws, scale_out=None):
    check(_lib.load().rvc_peak_normalize(_p(x), x.numel(), _p(ws), _p(scale_out), _stream()), "peak_normalize")
    return x


def change_rms(src, src64, out, hop, rate):
    """change_rms(audio, 16000, audio_opt, 16000, rate) (convert.py:150-152, :449) in place on the device
    output ``out`` [n]; src = the filtered 16 kHz input (f64 ``src64`` preferred, else f32 ``src``).
    The reference passes 16000 as both rates, so both envelopes use hop = 8000 (``hop``)."""
    lib = _lib.load()
    n_src = (src64 if src64 is not None else src).numel()
    n1, n2 = lib.rvc_rms_frames_len(n_src, hop), lib.rvc_rms_frames_len(out.numel(), hop)
    r1 = torch.empty(n1, device=out.device)
    r2 = torch.empty(n2, device=out.device)
    s64 = ctypes.c_void_p(src64.data_ptr()) if src64 is not None else None
    check(lib.rvc_rms_frames(s64, None if src64 is not None else _p(src), n_src, hop, _p(r1), _stream()),
          "rms_frames")
    check(lib.rvc_rms_frames(None, _p(out), out.numel(), hop, _p(r2), _stream()), "rms_frames")
    check(lib.rvc_rms_mix(_p(out), out.numel(), _p(r1), n1, _p(r2), n2, float(rate), _stream()), "rms_mix")
    return out


SQRT = math.sqrt
