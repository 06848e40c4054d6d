"""The model-level C ABI (include/rvc_amd.h "model-level API", csrc/rvc_model.cpp) from Python.

``NativeSynth`` is a drop-in ``net_g`` for ``VC.pipeline`` (convert.py:381, the ``.infer`` contract of
Synthesizer.infer, synthesizers.py:446-465) whose loader and launch sequence live in the library: the
checkpoint's weight dict goes in as named host arrays (``rvc_load_synth``, weight-norm folded natively),
``infer`` is one ``rvc_synth_infer`` call.  It is what a non-Python host (cgo / JNI / N-API)
binds; here it also pins the native sequence against ``SynthesizerAMD`` (tests/test_gpu_native.py).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check

PREC = {"fp32": 0, "bf16": 1, "bf16x3": 3, "fp32x6": 6, "f16x3": 16}


def synth_cfg(cpt: dict) -> "_lib.SynthCfg":
    """The checkpoint's "config" list (train.py:729-742) as rvc_synth_cfg (spk_embed_dim from emb_g,
    convert.py:558)."""
    cfg = list(cpt["config"])
    (_, _, inter, hidden, filt, n_heads, n_layers, ksz, _, _, rks, rds, ur, uic, uks, _, gin, sr) = cfg
    c = _lib.SynthCfg()
    c.inter_channels, c.hidden_channels, c.filter_channels = inter, hidden, filt
    c.n_heads, c.n_layers, c.kernel_size = n_heads, n_layers, ksz
    if len(rks) > 4 or len(ur) > 8 or any(len(d) > 4 for d in rds):
        raise ValueError("synth_cfg: more resblocks / dilations / upsamples than rvc_synth_cfg holds")
    c.n_resblocks, c.n_dilations = len(rks), len(rds[0])
    for j, (k, ds) in enumerate(zip(rks, rds)):
        c.resblock_kernel_sizes[j] = k
        for m, d in enumerate(ds):
            c.resblock_dilation_sizes[j][m] = d
    c.n_upsamples = len(ur)
    for i, (u, k) in enumerate(zip(ur, uks)):
        c.upsample_rates[i], c.upsample_kernel_sizes[i] = u, k
    c.upsample_initial_channel = uic
    c.spk_embed_dim = int(cpt["weight"]["emb_g.weight"].shape[0])
    c.gin_channels, c.sr = gin, sr
    return c


class NativeSynth:
    """Synthesizer.infer through rvc_ctx / rvc_load_synth / rvc_synth_infer.

    ``weights``: the checkpoint's weight dict as stored (fp16 weight_g / weight_v pairs, folded by the
    library) or any dict of already-folded fp32 tensors (synth.fold_weight_norm)."""

    def __init__(self, cpt: dict, device: str = "cuda", weights: dict | None = None, precision: str = "fp32"):
        self.lib = _lib.load()
        dev = torch.device(device)
        self.device = dev
        self.cfg = synth_cfg(cpt)
        self.upp = int(np.prod(cpt["config"][12]))
        self.inter = self.cfg.inter_channels
        ctx = ctypes.c_void_p()
        check(self.lib.rvc_ctx_create(dev.index or 0, ctypes.byref(ctx)), "rvc_ctx_create")
        self.ctx = ctx
        check(self.lib.rvc_ctx_set_precision(ctx, PREC[precision]), "rvc_ctx_set_precision")
        W = cpt["weight"] if weights is None else weights
        keep, params = [], (_lib.Param * len(W))()
        for i, (k, v) in enumerate(W.items()):
            a = v.detach().cpu().contiguous()
            if a.dtype not in (torch.float16, torch.float32):
                a = a.float()
            arr = np.ascontiguousarray(a.numpy())
            name = k.encode()
            keep += [arr, name]
            p = params[i]
            p.name, p.data = name, ctypes.c_void_p(arr.ctypes.data)
            p.dtype = 1 if arr.dtype == np.float16 else 0
            p.ndim = arr.ndim
            if not 1 <= arr.ndim <= 4:
                raise ValueError(f"NativeSynth: {k} has {arr.ndim} dims")
            for d, s in enumerate(arr.shape):
                p.shape[d] = s
        check(self.lib.rvc_load_synth(ctx, params, len(W), ctypes.byref(self.cfg)), "rvc_load_synth")
        del keep

    def __del__(self):
        ctx = getattr(self, "ctx", None)
        if ctx is not None and ctx.value:
            self.lib.rvc_ctx_destroy(ctx)
            self.ctx = None

    def out_len(self, T: int) -> int:
        return int(self.lib.rvc_synth_out_len(self.ctx, T))

    def infer(self, phone, phone_lengths, pitch=None, nsff0=None, sid=None, rate=None, z_noise=None,
              sine_noise=None, seed: int = 0):
        """Synthesizer.infer signature (synthesizers.py:446): phone [B, T, E] -> (o [B,1,L], x_mask, None).
        z_noise [B, inter, T] / sine_noise [B, T*upp(, 1)] inject the reference's draws; None = device Philox."""
        if rate is not None:
            raise NotImplementedError("rate (partial inference) is not used by VC.pipeline")
        if pitch is None or nsff0 is None:
            raise NotImplementedError("only f0 (NSF) models are on the hot path")
        B, T, E = phone.shape
        if torch.is_tensor(phone_lengths) and int(phone_lengths.reshape(-1).min()) != T:
            raise NotImplementedError("phone_lengths must equal the phone length (always true in VC.pipeline)")
        dev = self.device
        phone = phone.to(dev, torch.float32).contiguous()
        pitch = pitch.to(dev, torch.int64).reshape(B, T).contiguous()
        nsff0 = nsff0.to(dev, torch.float32).reshape(B, T).contiguous()
        sid_h = np.ascontiguousarray(
            (sid.reshape(-1).cpu().numpy() if torch.is_tensor(sid) else np.full(B, int(sid or 0))).astype(np.int64))
        if sid_h.size == 1 and B > 1:
            sid_h = np.full(B, int(sid_h[0]), np.int64)
        L = self.out_len(T)
        zn = z_noise.to(dev, torch.float32).reshape(B, self.inter, T).contiguous() if z_noise is not None else None
        sn = sine_noise.to(dev, torch.float32).reshape(B, L).contiguous() if sine_noise is not None else None
        o = torch.empty(B, 1, L, device=dev)
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        check(self.lib.rvc_synth_infer(self.ctx, p(phone), p(pitch), p(nsff0), B, T,
                                       ctypes.c_void_p(sid_h.ctypes.data), p(zn), p(sn), int(seed), p(o),
                                       ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "rvc_synth_infer")
        return o, torch.ones(B, 1, T, device=dev), None
