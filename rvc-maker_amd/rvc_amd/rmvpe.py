"""MI355X RMVPE f0 estimator: drop-in for ``RMVPE(model_path, is_half, device).infer_from_audio``
(main/library/predictors/RMVPE.py:183-226) as ``VC.get_f0_rmvpe`` uses it (convert.py:248-255).

Loaded once from an ``E2E(4, 1, (2, 2))`` state dict (the reference reloads ``rmvpe.pt`` on
every ``pipeline`` call, convert.py:251 -- this build keeps it resident).  BatchNorm is folded
into the convolutions on the host at load.  On the device:

  mel       stft_mag (reflect centre, Hann, f64 FFT in LDS, |X| rounded to f32 once)
            -> mel GEMM (513 -> 128) with log(clamp 1e-5) fused
  U-Net     images kept zero-bordered [C][H+2][W+2]; every 3x3 / 1x1 conv is the MFMA
            implicit-GEMM engine in 2-D mode (tap offsets + border masking), ReLU and the
            residual add fused; encoder skips are written straight into the decoder's concat
            buffers; ConvTranspose2d = 4 phase convs + interleave4
  head      cnn conv -> img_to_seq -> W_ih GEMM (both directions) -> bigru recurrence
            -> Linear 512->360 + sigmoid -> f64 decode + coarse pitch (rmvpe_decode)

Arithmetic (``precision``, RVC_RMVPE_PRECISION): "f64" (the default) runs every step above in f64 -- the convs on
the f64 matrix cores (rmvpe64.hip) -- except the BiGRU recurrence, which runs in f32 behind the f64 interface (f64
gate inputs and output; round 5: its decision noise is 1.8e-9 against the headline clip's smallest margin 3.2e-6,
profiles/r5_rmvpe_stage_prec.json; the all-f64 recurrence is ``rvc_bigru64_set_f32(0)`` / RVC_BIGRU64_F32=0) -- and
rounds only the salience to f32 for the decode.  RMVPE's f0 is a per-frame decision (argmax over 360 bins, 0.03 voicing threshold) and on the headline
clip the exact model's top two bins are 3.2e-6 apart at one frame, while every f32 evaluation errs by up to
1.7e-4 (the reference's own at other thread counts included): only an f64 network takes the exact model's
decisions everywhere.  "fp32sa" / any ops.PASSES name runs the f32 form (split-bf16 MFMA convs,
f32 BiGRU) for A/B comparisons.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import melbasis, ops
from .ops import ACT_LOGCLAMP, ACT_RELU, ACT_SIGMOID, pack_km

N_MELS, N_CLASS, NFFT, HOP = 128, 360, 1024, 160
EPS = 1e-5


# split-K target grid of the f32 form's convs (RVC_RMVPE_SPLITK; unset = the engine's default).  A Python-only
# diagnostic: the native rvc_rmvpe_forward does not read it, so setting it voids the native-vs-Python bit identity
# of the f32 form (the f64 form has its own split-K policy, RVC_C64_SPLITK_TILES, read by the library for both)
RMVPE_SPLITK = int(os.environ["RVC_RMVPE_SPLITK"]) if os.environ.get("RVC_RMVPE_SPLITK") else None


def _at_precision(fn):
    """Run a RMVPEAMD stage at the model's own arithmetic (self.precision) and split-K policy, whoever calls it
    (the f64 form has its own engine: the f32 engine's precision and split-K settings do not apply)."""
    def wrapped(self, *a, **k):
        if self.f64:
            return fn(self, *a, **k)
        with ops.precision(self.precision or ops.get_precision()), ops.splitk_target(RMVPE_SPLITK):
            return fn(self, *a, **k)
    wrapped.__name__, wrapped.__doc__ = fn.__name__, fn.__doc__
    return wrapped


def _fold_bn(sd, name):
    g, b = sd[name + ".weight"].double(), sd[name + ".bias"].double()
    m, v = sd[name + ".running_mean"].double(), sd[name + ".running_var"].double()
    s = g / torch.sqrt(v + EPS)
    return s, b - m * s


class _Conv2d:
    """3x3 (pad 1) or 1x1 conv on bordered images through the conv engine in 2-D mode: the f64 engine
    (conv64) or the f32 one (conv1d).  w / b come folded in f64."""

    def __init__(self, w, b, device, f64=True):
        Co, Ci, kh, kw = w.shape
        self.Co, self.Ci, self.k, self.f64 = Co, Ci, kh, f64
        self.v = None
        if f64:
            self.w = pack_km(w.reshape(Co, Ci, kh * kw).double()).to(device)
            self.b = b.double().to(device) if b is not None else None
            # the deep levels' 3x3 convs as Winograd F(4x4, 3x3) (rmvpe64.hip: 4x fewer f64 MFMA FLOPs)
            if kh == 3 and ops.wino64_use(Ci, Co):
                self.v = ops.wino64_weights(self.w, Ci, Co)
        else:
            self.w = pack_km(w.reshape(Co, Ci, kh * kw).float()).to(device)
            self.b = b.float().to(device) if b is not None else None
            self.wx, self.wx_nmf = ops.pack_x6(self.w, 1, Ci, kh * kw, Co)

    def __call__(self, x, H, W, out, **kw):
        """x / out: bordered images [C][H+2][W+2], or [B][C][H+2][W+2] views (batch strides from the views)."""
        wrap = W + 2
        L = (H + 2) * wrap
        if self.k == 3:
            toff = [dy * wrap + dx for dy in range(3) for dx in range(3)]
            pad = wrap + 1
        else:
            toff, pad = [0], 0
        if self.v is not None and ops.wino64_use(self.Ci, self.Co, H, W):
            return ops.wino64(x, self.v, self.Ci, self.Co, H, W, bias=self.b, out=out, **_batch_kw(x, out, kw), **kw)
        if self.f64:
            return ops.conv64(x, self.w, self.Ci, self.Co, self.k * self.k, bias=self.b, pad=pad, Lin=L, Lout=L,
                              out=out, toff=toff, wrap=wrap, **_batch_kw(x, out, kw), **kw)
        return ops.conv1d(x, self.w, self.Ci, self.Co, self.k * self.k, bias=self.b, pad=pad, Lin=L, Lout=L,
                          out=out, toff=toff, wrap=wrap, wx=self.wx, wx_nmf=self.wx_nmf, **_batch_kw(x, out, kw), **kw)


def _batch_kw(x, out, kw):
    """conv1d batch arguments for [B][C][H+2][W+2] image views (B = 1 for [C][H+2][W+2])."""
    if x.dim() != 4:
        return {"B": 1}
    res = kw.get("res")
    return {"B": x.shape[0], "x_bstride": x.stride(0), "y_bstride": out.stride(0),
            "res_bstride": res.stride(0) if res is not None else 0}


class _ConvT2d:
    """ConvTranspose2d(Ci, Co, 3, stride 2, padding 1, output_padding 1) + folded BN + ReLU as 4 phase convs."""

    # per output parity: list of (kernel index, source offset on the input grid)
    TAPS = {0: [(1, 0)], 1: [(0, 1), (2, 0)]}

    def __init__(self, w, scale, shift, device, f64=True):
        Ci, Co = w.shape[0], w.shape[1]
        self.Ci, self.Co, self.f64 = Ci, Co, f64
        wf = w.double() * scale.view(1, Co, 1, 1)
        self.bias = shift.double().to(device) if f64 else shift.float().to(device)
        self.phases = []
        for py in (0, 1):
            for px in (0, 1):
                taps = [(ky, kx, dy, dx) for ky, dy in self.TAPS[py] for kx, dx in self.TAPS[px]]
                wp = torch.stack([wf[:, :, ky, kx].t() for ky, kx, _, _ in taps], dim=-1)  # [Co, Ci, ntap]
                dyx = [(dy, dx) for _, _, dy, dx in taps]
                if f64:
                    self.phases.append((pack_km(wp).to(device), dyx, None, 0))
                else:
                    wkm = pack_km(wp.float()).to(device)
                    self.phases.append((wkm, dyx) + ops.pack_x6(wkm, 1, Ci, len(taps), Co))

    def __call__(self, x, H, W, out_cat):
        """x bordered [Ci][H+2][W+2] -> first Co channels of bordered out_cat [*][2H+2][2W+2]
        (or [B][...] views of both)."""
        wrap = W + 2
        L = (H + 2) * wrap
        B = x.shape[0] if x.dim() == 4 else None
        # the phase convs write the zero border
        ph = torch.empty((B or 1), 4, self.Co, H + 2, W + 2, device=x.device, dtype=x.dtype)
        for i, (wp, taps, wx, wx_nmf) in enumerate(self.phases):
            toff = [dy * wrap + dx for dy, dx in taps]
            out = ph[:, i] if B else ph[0, i]
            if self.f64:
                ops.conv64(x, wp, self.Ci, self.Co, len(taps), bias=self.bias, pad=0, Lin=L, Lout=L, out=out,
                           toff=toff, wrap=wrap, out_act=ACT_RELU, **_batch_kw(x, out, {}))
            else:
                ops.conv1d(x, wp, self.Ci, self.Co, len(taps), bias=self.bias, pad=0, Lin=L, Lout=L, out=out,
                           toff=toff, wrap=wrap, out_act=ACT_RELU, wx=wx, wx_nmf=wx_nmf, **_batch_kw(x, out, {}))
        if self.f64:
            ops.interleave4_64(ph if B else ph[0], out_cat, self.Co, H, W)
        else:
            for b in range(B or 1):
                ops.interleave4(ph[b], out_cat[b] if B else out_cat, self.Co, H, W)


class RMVPEAMD:
    def __init__(self, sd: dict, device: str = "cuda", n_blocks: int = 4, precision: str | None = None):
        dev = device
        self.device = dev
        self.nb = n_blocks
        # The f0 is a per-frame decision (argmax over 360 bins, voicing threshold): by default the whole network
        # runs in f64 (module note).  Any ops.PASSES name selects the f32 form at that conv arithmetic ("fp32sa":
        # 6-pass split-bf16 with split accumulators, round 3's default).
        self.precision = precision or os.environ.get("RVC_RMVPE_PRECISION", "f64")
        if self.precision != "f64" and self.precision not in ops.PASSES:
            raise ValueError(f"RMVPE precision must be 'f64' or one of {sorted(ops.PASSES)}")
        self.f64 = self.precision == "f64"
        f64 = self.f64
        self.dt = torch.float64 if f64 else torch.float32
        self.mel_basis = torch.from_numpy(melbasis.mel_filterbank(16000, NFFT, N_MELS, 30, 8000))
        self.window = torch.hann_window(NFFT).to(dev)  # float32 periodic, as RMVPE.py:166
        self.mel = (ops.Conv64 if f64 else ops.Conv)(self.mel_basis.unsqueeze(-1), None, device=dev)
        s, t = _fold_bn(sd, "unet.encoder.bn")
        self.in_scale, self.in_shift = (float(s[0]), float(t[0])) if f64 else \
            (float(s[0].float()), float(t[0].float()))

        def cbr(p):
            out = {}
            for conv, bn in (("conv.0", "conv.1"), ("conv.3", "conv.4")):
                sc, sh = _fold_bn(sd, f"{p}.{bn}")
                w = sd[f"{p}.{conv}.weight"].double() * sc.view(-1, 1, 1, 1)
                out[conv] = _Conv2d(w if f64 else w.float(), sh if f64 else sh.float(), dev, f64)
            if f"{p}.shortcut.weight" in sd:
                out["sc"] = _Conv2d(sd[f"{p}.shortcut.weight"], sd[f"{p}.shortcut.bias"], dev, f64)
            return out

        self.enc = [[cbr(f"unet.encoder.layers.{l}.conv.{b}") for b in range(n_blocks)] for l in range(5)]
        self.inter = [[cbr(f"unet.intermediate.layers.{l}.conv.{b}") for b in range(n_blocks)]
                      for l in range(4)]
        self.dec = []
        for l in range(5):
            p = f"unet.decoder.layers.{l}"
            sc, sh = _fold_bn(sd, p + ".conv1.1")
            self.dec.append((_ConvT2d(sd[p + ".conv1.0.weight"], sc, sh, dev, f64),
                             [cbr(f"{p}.conv2.{b}") for b in range(n_blocks)]))
        self.cnn = _Conv2d(sd["cnn.weight"], sd["cnn.bias"], dev, f64)
        g = "fc.0.gru."
        Lin = ops.Conv64 if f64 else ops.Conv
        self.w_ih = Lin(torch.cat([sd[g + "weight_ih_l0"], sd[g + "weight_ih_l0_reverse"]], 0).unsqueeze(-1),
                        torch.cat([sd[g + "bias_ih_l0"], sd[g + "bias_ih_l0_reverse"]], 0), device=dev)
        self.w_hh = torch.stack([sd[g + "weight_hh_l0"], sd[g + "weight_hh_l0_reverse"]], 0).to(self.dt).contiguous().to(dev)
        self.b_hh = torch.stack([sd[g + "bias_hh_l0"], sd[g + "bias_hh_l0_reverse"]], 0).to(self.dt).contiguous().to(dev)
        self.fc = Lin(sd["fc.1.weight"].unsqueeze(-1), sd["fc.1.bias"], device=dev)
        self.gran_words = ops.GRU64_GRAN if f64 else 1024  # BiGRU hand-off scratch per sequence (int64 words)
        self.gran = torch.zeros(self.gran_words, dtype=torch.int64, device=dev)  # the default stream's
        self._grans = {}
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)

    @classmethod
    def from_file(cls, path, device="cuda"):
        return cls(torch.load(path, map_location="cpu", weights_only=True), device)

    # ------------------------------------------------------------------ pieces
    @_at_precision
    def mel_spectrogram(self, audio: torch.Tensor) -> torch.Tensor:
        """MelSpectrogram.forward (RMVPE.py:162-181): audio [N] f32 -> log-mel [128][F] (f64 in the f64 form)."""
        N = audio.numel()
        F = 1 + N // HOP
        mag = torch.empty(NFFT // 2 + 1, F, device=audio.device, dtype=self.dt)
        (ops.stft_mag64 if self.f64 else ops.stft_mag)(audio, self.window, mag, N, F, NFFT, HOP)
        return self.mel(mag, out_act=ACT_LOGCLAMP, out_slope=1e-5)

    @_at_precision
    def mel_spectrogram_batch(self, xb: torch.Tensor) -> torch.Tensor:
        """B equal-length signals [B][N] -> log-mel [B][128][F] (the GEMMs batched, framing per signal)."""
        B, N = xb.shape
        F = 1 + N // HOP
        mag = torch.empty(B, NFFT // 2 + 1, F, device=xb.device, dtype=self.dt)
        (ops.stft_mag64 if self.f64 else ops.stft_mag)(xb, self.window, mag, N, F, NFFT, HOP)
        return self.mel(mag, out_act=ACT_LOGCLAMP, out_slope=1e-5)

    def _cbr(self, blk, x, H, W, out):
        dev = x.device
        Co = blk["conv.0"].Co
        bshape = (x.shape[0],) if x.dim() == 4 else ()
        # 2-D convs cover the whole bordered image and write its border as 0: no zero-fill needed
        h = torch.empty(*bshape, Co, H + 2, W + 2, device=dev, dtype=self.dt)
        blk["conv.0"](x, H, W, h, out_act=ACT_RELU)
        if "sc" in blk:
            sc = torch.empty(*bshape, Co, H + 2, W + 2, device=dev, dtype=self.dt)
            blk["sc"](x, H, W, sc)
            res = sc
        else:
            res = x
        blk["conv.3"](h, H, W, out, out_act=ACT_RELU, res=res)
        return out

    def mel_image(self, mel: torch.Tensor) -> tuple[torch.Tensor, int]:
        """mel2hidden's input (RMVPE.py:210-213): mel [128][F] -> bordered image [1][Tp+2][130] (reflect-padded
        to Tp = F rounded up to 32, input BatchNorm applied), Tp."""
        F = mel.shape[-1]
        Tp = 32 * ((F - 1) // 32 + 1)
        mel = mel.to(self.dt).contiguous()  # a caller's f32 mel (the reference's mel2hidden input) in the f64 form
        # (the f64 kernels write the zero border themselves: no zero-fill launch on the f0 chain)
        x = (torch.empty if self.f64 else torch.zeros)(1, Tp + 2, N_MELS + 2, device=mel.device, dtype=self.dt)
        (ops.mel_image64 if self.f64 else ops.mel_image)(mel, x, N_MELS, F, Tp, self.in_scale, self.in_shift)
        return x, Tp

    def _pool(self, x, pooled, C, H, W):
        if self.f64:
            ops.avgpool2_64(x, pooled, C, H, W)
        elif x.dim() == 4:
            for b in range(x.shape[0]):
                ops.avgpool2(x[b], pooled[b], C, H, W)
        else:
            ops.avgpool2(x, pooled, C, H, W)

    def _to_seq(self, img, seq, H, W):
        if self.f64:
            ops.img_to_seq64(img, seq, 3, H, W)
        elif img.dim() == 4:
            for b in range(img.shape[0]):
                ops.img_to_seq(img[b], seq[b], 3, H, W)
        else:
            ops.img_to_seq(img, seq, 3, H, W)

    def _unet(self, x, H, bshape):
        """E2E up to the GRU input on bordered images x [(B)][1][H+2][130] -> cnn head rows [(B)][384][H]."""
        dev = x.device
        W = N_MELS
        cats = []
        C = 16
        for l in range(5):
            # cat[C:] is written whole by the encoder's last conv (border included), cat[:C] by the decoder's
            # interleave (which writes its border in the f64 form); pooled by the f64 pooling, border included
            alloc = torch.empty if self.f64 else torch.zeros
            cat = alloc(*bshape, 2 * C, H + 2, W + 2, device=dev, dtype=self.dt)
            for b, blk in enumerate(self.enc[l]):
                out = cat[..., C:, :, :] if b == self.nb - 1 else \
                    torch.empty(*bshape, C, H + 2, W + 2, device=dev, dtype=self.dt)
                x = self._cbr(blk, x, H, W, out)
            cats.append((cat, C, H, W))
            pooled = alloc(*bshape, C, H // 2 + 2, W // 2 + 2, device=dev, dtype=self.dt)
            self._pool(x, pooled, C, H, W)
            x, H, W = pooled, H // 2, W // 2
            C *= 2
        for layer in self.inter:
            for blk in layer:
                x = self._cbr(blk, x, H, W, torch.empty(*bshape, blk["conv.0"].Co, H + 2, W + 2, device=dev,
                                                        dtype=self.dt))
        for i, (convt, blocks) in enumerate(self.dec):
            cat, C, Ho, Wo = cats[-1 - i]
            convt(x, H, W, cat)
            x, H, W = cat, Ho, Wo
            for blk in blocks:
                x = self._cbr(blk, x, H, W, torch.empty(*bshape, blk["conv.0"].Co, H + 2, W + 2, device=dev,
                                                        dtype=self.dt))
        img = torch.empty(*bshape, 3, H + 2, W + 2, device=dev, dtype=self.dt)
        self.cnn(x, H, W, img)
        seq = torch.empty(*bshape, 3 * W, H, device=dev, dtype=self.dt)
        self._to_seq(img, seq, H, W)
        return seq

    @_at_precision
    def unet_seq(self, x: torch.Tensor, H: int) -> torch.Tensor:
        """E2E up to the GRU input (RMVPE.py:143-144, 254): bordered image [1][H+2][130] (H % 32 == 0)
        -> cnn head rows [384][H]."""
        return self._unet(x, H, ())

    def gran_ws(self, n: int = 1) -> torch.Tensor:
        """BiGRU hand-off scratch for ``n`` sequences on the current stream: recurrences running at once on
        different streams (the clip stream's alternating front pipelines) must not share one."""
        n *= self.gran_words
        s = torch.cuda.current_stream(self.device)
        if s == torch.cuda.default_stream(self.device) and n <= self.gran.numel():
            return self.gran
        key = s.stream_id
        g = self._grans.get(key)
        if g is None or g.numel() < n:
            g = torch.zeros(n, dtype=torch.int64, device=self.device)
            self._grans[key] = g
        return g

    def _head(self, seq, B, Tp):
        """W_ih GEMM -> BiGRU (B recurrences side by side) -> Linear + sigmoid: seq [(B)][384][Tp] ->
        salience [(B)][360][Tp] f32."""
        gi = self.w_ih(seq)  # [(B)][1536][Tp]
        y = torch.empty(*((B,) if seq.dim() == 3 else ()), 512, Tp, device=seq.device, dtype=self.dt)
        gran = self.gran_ws(min(B, ops.GRU_B_MAX))
        if self.f64:
            ops.bigru64_batched(gi, self.w_hh, self.b_hh, y, gran, self.err, B, Tp)
            return self.fc(y, out_act=ACT_SIGMOID, out_f32=True)
        if seq.dim() == 3:
            ops.bigru_batched(gi, self.w_hh, self.b_hh, y, gran, self.err, B, Tp)
        else:
            ops.bigru(gi, self.w_hh, self.b_hh, y, gran, self.err, Tp)
        return self.fc(y, out_act=ACT_SIGMOID)

    @_at_precision
    def head(self, seq: torch.Tensor) -> torch.Tensor:
        """BiGRU + Linear + Sigmoid (RMVPE.py:254-260, 141): seq [384][Tp] -> salience [360][Tp] (f32)."""
        return self._head(seq, 1, seq.shape[-1])

    @_at_precision
    def salience(self, mel: torch.Tensor) -> tuple[torch.Tensor, int]:
        """mel2hidden + E2E (RMVPE.py:210-215, 143-144): mel [128][F] -> salience [360][Tp] (Tp = F rounded up to 32)."""
        x, Tp = self.mel_image(mel)
        return self.head(self.unet_seq(x, Tp)), Tp

    def decode(self, sal, Tp, F, thred=0.03, pitch_shift=0.0, want_f0=False, post=None):
        """rmvpe_decode over the first F frames of salience [360][Tp] -> (coarse, pitchf, f0 | None)."""
        dev = sal.device
        coarse = torch.empty(F, dtype=torch.int64, device=dev)
        pitchf = torch.empty(F, device=dev)
        f0 = torch.empty(F, dtype=torch.float64, device=dev) if want_f0 else None
        ops.rmvpe_decode(sal, Tp, F, thred, math.pow(2, pitch_shift / 12), f0, coarse, pitchf, post)
        return coarse, pitchf, f0

    @_at_precision
    def salience_batch(self, mel: torch.Tensor) -> tuple[torch.Tensor, int]:
        """salience for B clips at once: mel [B][128][F] -> [B][360][Tp].  Every conv of the U-Net, the
        W_ih / fc GEMMs and the BiGRU (B recurrences side by side) run batched (and in the f64 form the image
        glue kernels too)."""
        dev = mel.device
        B, _, F = mel.shape
        Tp = 32 * ((F - 1) // 32 + 1)
        mel = mel.to(self.dt).contiguous()
        x = (torch.empty if self.f64 else torch.zeros)(B, 1, Tp + 2, N_MELS + 2, device=dev, dtype=self.dt)
        if self.f64:
            ops.mel_image64(mel, x, N_MELS, F, Tp, self.in_scale, self.in_shift)
        else:
            for b in range(B):
                ops.mel_image(mel[b], x[b], N_MELS, F, Tp, self.in_scale, self.in_shift)
        seq = self._unet(x, Tp, (B,))
        return self._head(seq, B, Tp), Tp

    def f0_device_batch(self, xb: torch.Tensor, thred: float = 0.03, pitch_shift: float = 0.0, post=None,
                        want_f0=False, want_salience=False):
        """B equal-length signals [B][N] -> (coarse int64 [B][F], pitchf f32 [B][F]) [+ raw f0 f64 [B][F]]
        [+ salience [B][360][Tp]]; same per-clip result as ``f0_device`` up to the summation order of the batched
        GEMMs (split-K follows the batched grid)."""
        mel = self.mel_spectrogram_batch(xb)
        B, _, F = mel.shape
        sal, Tp = self.salience_batch(mel)
        coarse = torch.empty(B, F, dtype=torch.int64, device=xb.device)
        pitchf = torch.empty(B, F, device=xb.device)
        f0 = torch.empty(B, F, dtype=torch.float64, device=xb.device) if want_f0 else None
        for b in range(B):
            ops.rmvpe_decode(sal[b], Tp, F, thred, math.pow(2, pitch_shift / 12), f0[b] if want_f0 else None,
                             coarse[b], pitchf[b], post)
        out = (coarse, pitchf) + ((f0,) if want_f0 else ()) + ((sal,) if want_salience else ())
        return out

    def f0_device(self, audio: torch.Tensor, thred: float = 0.03, pitch_shift: float = 0.0, want_f0=False,
                  post=None):
        """audio [N] f32 device -> (coarse int64 [F], pitchf f32 [F], f0 f64 [F] | None) on the device;
        ``post`` (ops.F0Post) adds get_f0's autotune / f0-file steps."""
        mel = self.mel_spectrogram(audio)
        F = mel.shape[-1]
        sal, Tp = self.salience(mel)
        return self.decode(sal, Tp, F, thred, pitch_shift, want_f0, post)

    def check_error(self):
        """Raise if a BiGRU launch since the last check timed out (its f0 is then garbage); clears the flag."""
        if int(self.err.item()) != 0:
            self.err.zero_()
            raise RuntimeError("rvc_amd: bigru recurrence timed out (granule hand-off stalled); f0 invalid")

    # ------------------------------------------------------------------ reference API
    def infer_from_audio(self, audio: np.ndarray, thred: float = 0.03) -> np.ndarray:
        """RMVPE.infer_from_audio (RMVPE.py:223-226): f64 numpy [N] -> f64 numpy f0 [1 + N//160]."""
        x = torch.from_numpy(np.asarray(audio)).float().to(self.device)
        _, _, f0 = self.f0_device(x, thred, 0.0, want_f0=True)
        out = f0.cpu().numpy()
        self.check_error()
        return out
