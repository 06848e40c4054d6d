"""The model-level C ABI (include/rvc_amd.h "model-level API", csrc/rvc_model.cpp, csrc/rvc_frontend.cpp)
from Python.

``NativeSynth`` is a drop-in ``net_g`` for ``VC.pipeline`` (convert.py:381, the ``.infer`` contract of
Synthesizer.infer, synthesizers.py:446-465) whose loader and launch sequence live in the library: the
checkpoint's weight dict goes in as named host arrays (``rvc_load_synth``, weight-norm folded natively),
``infer`` is one ``rvc_synth_infer`` call.  It is what a non-Python host (cgo / JNI / N-API)
binds; here it also pins the native sequence against ``SynthesizerAMD`` (tests/test_gpu_native.py).
``NativeContentVec`` (``model.extract_features``, fairseq.py:1459) and ``NativeRMVPE``
(``RMVPE.infer_from_audio``, RMVPE.py:223-226) do the same for the front end; each owns its own
``rvc_ctx``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import check

PREC = {"fp32": 0, "bf16": 1, "bf16x3": 3, "fp32x6": 6, "fp32sa": 7, "f16x3": 16, "f64": 64}


def _rmvpe_precision(name):
    """RMVPE's arithmetic as RMVPEAMD picks it (RVC_RMVPE_PRECISION, default "f64")."""
    return PREC[name or os.environ.get("RVC_RMVPE_PRECISION", "f64")]


def _params(W: dict):
    """Named host arrays (rvc_param) for a weight dict; returns (params, keep-alive list)."""
    keep, params = [], (_lib.Param * len(W))()
    for i, (k, v) in enumerate(W.items()):
        a = torch.as_tensor(v).detach().cpu().contiguous()
        if a.dtype not in (torch.float16, torch.float32, torch.float64):
            a = a.float()
        arr = np.ascontiguousarray(a.numpy())
        if not 1 <= arr.ndim <= 4:
            raise ValueError(f"rvc_param: {k} has {arr.ndim} dims")
        name = k.encode()
        keep += [arr, name]
        p = params[i]
        p.name, p.data = name, ctypes.c_void_p(arr.ctypes.data)
        p.dtype = {np.dtype(np.float16): 1, np.dtype(np.float64): 2}.get(arr.dtype, 0)
        p.ndim = arr.ndim
        for d, s in enumerate(arr.shape):
            p.shape[d] = s
    return params, keep


def export_synth_safetensors(cpt: dict, path: str) -> None:
    """The .pth's "weight" dict, unchanged (fp16 weight_g / weight_v pairs), as a safetensors file with
    __metadata__["rvc_synth_cfg"] = the rvc_synth_cfg ints in field order: what a non-Python host
    (examples/c_host/synth_demo.c) loads and hands to rvc_load_synth."""
    from safetensors.torch import save_file
    ints = np.frombuffer(bytes(synth_cfg(cpt)), dtype=np.int32)
    save_file({k: v.detach().cpu().contiguous() for k, v in cpt["weight"].items()}, path,
              metadata={"rvc_synth_cfg": " ".join(str(int(i)) for i in ints)})


def export_safetensors(tensors: dict, path: str, **meta_ints) -> None:
    """Floating tensors of a checkpoint dict as safetensors, with each keyword as a __metadata__ string of
    ints: e.g. the ContentVec ``model`` dict with rvc_contentvec_cfg=[768, 12, 16, 0] (examples/c_host)."""
    from safetensors.torch import save_file
    W = {k: v.detach().cpu().contiguous() for k, v in tensors.items() if torch.is_tensor(v) and v.is_floating_point()}
    save_file(W, path, metadata={k: " ".join(str(int(i)) for i in v) for k, v in meta_ints.items()})


class _Ctx:
    """One rvc_ctx on a device (destroyed with the object)."""

    def __init__(self, device, precision="fp32"):
        self.lib = _lib.load()
        self.device = torch.device(device)
        ctx = ctypes.c_void_p()
        check(self.lib.rvc_ctx_create(self.device.index or 0, ctypes.byref(ctx)), "rvc_ctx_create")
        self.ctx = ctx
        check(self.lib.rvc_ctx_set_precision(ctx, PREC[precision]), "rvc_ctx_set_precision")

    def __del__(self):
        ctx = getattr(self, "ctx", None)
        if ctx is not None and ctx.value:
            self.lib.rvc_ctx_destroy(ctx)
            self.ctx = None

    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)


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


class NativeSynth(_Ctx):
    """Synthesizer.infer through rvc_ctx / rvc_load_synth / rvc_synth_infer.

    ``weights``: the checkpoint's weight dict as stored (fp16 weight_g / weight_v pairs, folded by the
    library) or any dict of already-folded fp32 tensors (synth.fold_weight_norm)."""

    def __init__(self, cpt: dict, device: str = "cuda", weights: dict | None = None, precision: str = "fp32"):
        super().__init__(device, precision)
        self.cfg = synth_cfg(cpt)
        self.upp = int(np.prod(cpt["config"][12]))
        self.inter = self.cfg.inter_channels
        W = cpt["weight"] if weights is None else weights
        params, keep = _params(W)
        check(self.lib.rvc_load_synth(self.ctx, params, len(W), ctypes.byref(self.cfg)), "rvc_load_synth")
        del keep

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
                                       self.stream()), "rvc_synth_infer")
        return o, torch.ones(B, 1, T, device=dev), None


class NativeContentVec(_Ctx):
    """HubertModel.extract_features through rvc_load_contentvec / rvc_contentvec_forward."""

    def __init__(self, ckpt: dict, device: str = "cuda", precision: str = "fp32", weights: dict | None = None):
        """``weights``: a replacement for ckpt["model"] (e.g. with encoder.pos_conv already folded)."""
        super().__init__(device, precision)
        cfg = ckpt["cfg"]["model"]
        if cfg.get("extractor_mode", "default") != "default" or cfg.get("layer_norm_first", False):
            raise NotImplementedError("ContentVec/HuBERT-base layout only (extractor 'default', post-LN)")
        c = _lib.ContentVecCfg()
        c.encoder_embed_dim = cfg.get("encoder_embed_dim", 768)
        c.encoder_attention_heads = cfg.get("encoder_attention_heads", 12)
        c.conv_pos_groups = cfg.get("conv_pos_groups", 16)
        self.E = c.encoder_embed_dim
        sd = ckpt["model"] if weights is None else weights
        W = {k: v for k, v in sd.items() if torch.is_tensor(v) and v.is_floating_point()}
        params, keep = _params(W)
        check(self.lib.rvc_load_contentvec(self.ctx, params, len(W), ctypes.byref(c)), "rvc_load_contentvec")
        self.proj_dim = int(W["final_proj.weight"].shape[0])
        del keep

    def frames(self, n: int) -> int:
        return int(self.lib.rvc_contentvec_frames(n))

    def forward(self, wav, output_layer: int = 12, final_proj: bool = False):
        """wav [B, N] or [N] f32 (device) -> feats [B, T, C] (C = 768, or final_proj's width)."""
        wav = wav.to(self.device, torch.float32)
        wav = wav.reshape(1, -1) if wav.dim() == 1 else wav
        wav = wav.contiguous()
        B, N = wav.shape
        T = self.frames(N)
        out = torch.empty(B, T, self.proj_dim if final_proj else self.E, device=self.device)
        check(self.lib.rvc_contentvec_forward(self.ctx, ctypes.c_void_p(wav.data_ptr()), B, N, int(output_layer),
                                              int(bool(final_proj)), ctypes.c_void_p(out.data_ptr()), self.stream()),
              "rvc_contentvec_forward")
        return out

    def extract_features(self, source, padding_mask=None, mask=False, ret_conv=False, output_layer=None):
        """fairseq.py:1459: source [1, N] -> (x [1, T_f, 768], padding_mask [1, T_f])."""
        if padding_mask is not None and bool(padding_mask.any()):
            raise NotImplementedError("padded sources are not on the hot path (VC passes an all-False mask)")
        x = self.forward(source, output_layer or 12)
        return x, torch.zeros(x.shape[0], x.shape[1], dtype=torch.bool, device=x.device)


class NativeRMVPE(_Ctx):
    """RMVPE salience / f0 through rvc_load_rmvpe / rvc_rmvpe_forward / rvc_rmvpe_decode."""

    def __init__(self, sd: dict, device: str = "cuda", window=None, mel_basis=None, rmvpe_precision=None):
        super().__init__(device)
        check(self.lib.rvc_ctx_set_rmvpe_precision(self.ctx, _rmvpe_precision(rmvpe_precision)),
              "rvc_ctx_set_rmvpe_precision")
        W = dict(sd)
        if window is not None:
            W["window"] = window
        if mel_basis is not None:
            W["mel_basis"] = mel_basis
        W = {k: v for k, v in W.items() if torch.as_tensor(v).is_floating_point()}
        params, keep = _params(W)
        check(self.lib.rvc_load_rmvpe(self.ctx, params, len(W)), "rvc_load_rmvpe")
        del keep

    def salience(self, wav):
        """wav [B, N] or [N] f32 (device) -> (salience [B, 360, Tp], F)."""
        wav = wav.to(self.device, torch.float32)
        wav = (wav.reshape(1, -1) if wav.dim() == 1 else wav).contiguous()
        B, N = wav.shape
        Tp, F = int(self.lib.rvc_rmvpe_salience_ld(N)), int(self.lib.rvc_rmvpe_frames(N))
        sal = torch.empty(B, 360, Tp, device=self.device)
        check(self.lib.rvc_rmvpe_forward(self.ctx, ctypes.c_void_p(wav.data_ptr()), B, N,
                                         ctypes.c_void_p(sal.data_ptr()), self.stream()), "rvc_rmvpe_forward")
        return sal, F

    def check(self):
        check(self.lib.rvc_rmvpe_check(self.ctx), "rvc_rmvpe_check")

    def infer_from_audio(self, audio, thred: float = 0.03) -> np.ndarray:
        """RMVPE.infer_from_audio (RMVPE.py:223-226): f64 numpy [N] -> f64 numpy f0 [1 + N//160]."""
        from . import ops
        x = torch.from_numpy(np.asarray(audio)).float().to(self.device)
        sal, F = self.salience(x)
        Tp = sal.shape[-1]
        f0 = torch.empty(F, dtype=torch.float64, device=self.device)
        coarse = torch.empty(F, dtype=torch.int64, device=self.device)
        pitchf = torch.empty(F, device=self.device)
        ops.rmvpe_decode(sal[0], Tp, F, thred, 1.0, f0, coarse, pitchf)
        out = f0.cpu().numpy()
        self.check()
        return out


class NativeCrepe(_Ctx):
    """VC.get_f0_crepe + get_f0's quantiser through rvc_load_crepe / rvc_crepe_f0."""

    def __init__(self, sd: dict, device: str = "cuda", precision: str = "fp32", log_trans=None, bn=None):
        """``bn``: optional [(alpha, beta)] x 6 folded BatchNorms (CrepeAMD.bns) instead of the library's fold."""
        super().__init__(device, precision)
        W = {k: v for k, v in sd.items() if torch.as_tensor(v).is_floating_point()}
        for i, (a, b) in enumerate(bn or []):
            W[f"conv{i + 1}_BN.alpha"], W[f"conv{i + 1}_BN.beta"] = a.cpu(), b.cpu()
        if log_trans is not None:
            W["log_trans"] = torch.as_tensor(log_trans, dtype=torch.float64)
        params, keep = _params(W)
        check(self.lib.rvc_load_crepe(self.ctx, params, len(W)), "rvc_load_crepe")
        del keep

    def f0_device(self, audio, pitch_shift: float = 0.0, dither=None, seed: int = 0, want_probs: bool = False):
        """audio [N] f32 (device) -> (coarse int64 [T], pitchf f32 [T], probs [360][T] | None)."""
        audio = audio.to(self.device, torch.float32).reshape(-1).contiguous()
        N = audio.numel()
        T = 1 + N // 160
        coarse = torch.empty(T, dtype=torch.int64, device=self.device)
        pitchf = torch.empty(T, device=self.device)
        probs = torch.empty(360, T, device=self.device) if want_probs else None
        d = None
        if dither is not None:
            d = torch.as_tensor(np.asarray(dither, dtype=np.float32)).to(self.device).contiguous()
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        check(self.lib.rvc_crepe_f0(self.ctx, p(audio), N, p(d), int(seed), float(pitch_shift), None, p(probs),
                                    p(coarse), p(pitchf), self.stream()), "rvc_crepe_f0")
        return coarse, pitchf, probs


class NativeVC(_Ctx):
    """One ``VC.pipeline`` segment through the model-level ABI: ContentVec, RMVPE and the synthesizer loaded on
    one context, ``convert`` = rvc_vc_convert (filtfilt, f0, features, upsample + protect, synthesizer, trim,
    peak normalisation).  ``synth_weights`` / ``hub_weights`` / ``rmvpe_consts`` as the single-model classes."""

    def __init__(self, hub_ckpt: dict, rmvpe_sd: dict, synth_cpt: dict, device: str = "cuda", precision="fp32",
                 synth_weights=None, hub_weights=None, window=None, mel_basis=None, rmvpe_precision=None):
        super().__init__(device, precision)
        check(self.lib.rvc_ctx_set_rmvpe_precision(self.ctx, _rmvpe_precision(rmvpe_precision)),
              "rvc_ctx_set_rmvpe_precision")
        cfg = hub_ckpt["cfg"]["model"]
        c = _lib.ContentVecCfg()
        c.encoder_embed_dim = cfg.get("encoder_embed_dim", 768)
        c.encoder_attention_heads = cfg.get("encoder_attention_heads", 12)
        c.conv_pos_groups = cfg.get("conv_pos_groups", 16)
        sd = hub_ckpt["model"] if hub_weights is None else hub_weights
        W = {k: v for k, v in sd.items() if torch.is_tensor(v) and v.is_floating_point()}
        params, keep = _params(W)
        check(self.lib.rvc_load_contentvec(self.ctx, params, len(W), ctypes.byref(c)), "rvc_load_contentvec")
        W = dict(rmvpe_sd)
        if window is not None:
            W["window"] = window
        if mel_basis is not None:
            W["mel_basis"] = mel_basis
        W = {k: v for k, v in W.items() if torch.as_tensor(v).is_floating_point()}
        params, keep = _params(W)
        check(self.lib.rvc_load_rmvpe(self.ctx, params, len(W)), "rvc_load_rmvpe")
        self.cfg = synth_cfg(synth_cpt)
        W = synth_cpt["weight"] if synth_weights is None else synth_weights
        params, keep = _params(W)
        check(self.lib.rvc_load_synth(self.ctx, params, len(W), ctypes.byref(self.cfg)), "rvc_load_synth")
        del keep
        self.tgt_sr = int(synth_cpt["config"][-1])

    def load_index(self, index) -> None:
        """A faiss_index.IVFFlatIndex (as read_index gives it) -> rvc_load_index."""
        sizes = np.array([len(i) for i in index.ids], dtype=np.int64)
        off = np.zeros(index.nlist + 1, dtype=np.int64)
        np.cumsum(sizes, out=off[1:])
        keep = [np.ascontiguousarray(index.centroids, dtype=np.float32), off,
                np.ascontiguousarray(np.concatenate(index.codes) if off[-1] else np.zeros((1, index.d)), np.float32),
                np.ascontiguousarray(np.concatenate(index.ids) if off[-1] else np.zeros(1), np.int64),
                np.ascontiguousarray(index.reconstruct_n(0, index.ntotal), np.float32)]
        x = _lib.IvfIndex()
        x.d, x.nlist, x.ntotal, x.nprobe = index.d, index.nlist, int(off[-1]), index.nprobe
        x.centroids, x.list_off, x.codes, x.ids, x.big = (ctypes.c_void_p(a.ctypes.data) for a in keep)
        check(self.lib.rvc_load_index(self.ctx, ctypes.byref(x)), "rvc_load_index")

    def args(self, sid=0, pitch=0.0, protect=0.33, version="v2", seed=0, x_pad=1, x_max=41, index_rate=0.0):
        a = _lib.VcArgs()
        a.index_rate = float(index_rate)
        a.sid, a.pitch_shift, a.protect, a.version = int(sid), float(pitch), float(protect), 1 if version == "v1" else 2
        a.x_pad, a.x_max, a.tgt_sr, a.seed = x_pad, x_max, self.tgt_sr, int(seed)
        return a

    F0_METHODS = {"rmvpe": 0, "crepe": 1, "pm": 2}

    def convert(self, audio, sid=0, pitch=0.0, protect=0.33, version="v2", seed=0, index_rate=0.0, f0_method="rmvpe",
                f0_autotune=False, f0_autotune_strength=1.0, inp_f0=None, volume_envelope=1.0, crepe_dither=None):
        """audio f32 [N] 16 kHz (device) -> waveform f32 at tgt_sr (device): rvc_vc_convert_ex, i.e. the whole
        VC.pipeline (segmentation of inputs over 41 s, f0 method, autotune, f0 file rows ``inp_f0`` f32 [n][2] as
        read_f0_file gives them, volume envelope); CREPE (``f0_method="crepe"``, loaded with load_crepe) takes its
        dither from ``crepe_dither`` (device f32 [1 + padded N // 160]) or draws it on the device from seed."""
        audio = audio.to(self.device, torch.float32).reshape(-1).contiguous()
        a = self.args(sid, pitch, protect, version, seed, index_rate=index_rate)
        o = _lib.VcOpts()
        o.f0_method = self.F0_METHODS[f0_method]
        o.f0_autotune, o.f0_autotune_strength = int(bool(f0_autotune)), float(f0_autotune_strength)
        keep = None
        if inp_f0 is not None:
            keep = np.ascontiguousarray(inp_f0, dtype=np.float32)
            o.f0_file, o.f0_file_rows = ctypes.c_void_p(keep.ctypes.data), keep.shape[0]
        o.volume_envelope = float(volume_envelope)
        if crepe_dither is not None:
            o.crepe_dither = ctypes.c_void_p(crepe_dither.data_ptr())
        cap = int(self.lib.rvc_vc_out_len(self.ctx, audio.numel(), ctypes.byref(a)))
        if cap <= 0:
            raise RuntimeError(f"rvc_vc_out_len: {self.lib.rvc_last_error().decode()}")
        out = torch.empty(cap, device=self.device)
        n = ctypes.c_int64(0)
        check(self.lib.rvc_vc_convert_ex(self.ctx, ctypes.c_void_p(audio.data_ptr()), audio.numel(), ctypes.byref(a),
                                         ctypes.byref(o), ctypes.c_void_p(out.data_ptr()), cap, ctypes.byref(n),
                                         self.stream()), "rvc_vc_convert_ex")
        del keep
        return out[: n.value]

    def load_crepe(self, sd: dict, log_trans=None, bn=None) -> None:
        """A CREPE state dict (any capacity) for f0_method="crepe" (rvc_load_crepe; optional f64 log_trans and
        [(alpha, beta)] x 6 folded BatchNorms, as NativeCrepe takes them)."""
        W = {k: v for k, v in sd.items() if torch.as_tensor(v).is_floating_point()}
        if log_trans is not None:
            W["log_trans"] = torch.as_tensor(log_trans, dtype=torch.float64)
        for i, (al, be) in enumerate(bn or []):
            W[f"conv{i + 1}_BN.alpha"], W[f"conv{i + 1}_BN.beta"] = al.cpu(), be.cpu()
        params, keep = _params(W)
        check(self.lib.rvc_load_crepe(self.ctx, params, len(W)), "rvc_load_crepe")
        del keep
