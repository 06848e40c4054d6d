"""MI355X CREPE f0: drop-in for ``VC.get_f0_crepe`` (main/inference/convert.py:230-237) and the
``get_f0`` coarse-pitch step that follows it (convert.py:304-323), for every capacity
(tiny .. full) of ``main/library/predictors/CREPE.py``.

  frames      rvc_crepe_frames: 1024-sample frames at hop 160, zero-mean / unit-std (CREPE.py:151-171)
  network     6 x [conv (k x 1) on the conv engine with ReLU fused, rvc_bn_maxpool], the last layer
              written straight into the classifier's (position, channel) flatten order, then the
              Linear(in_features, 360) as a K=1 conv with sigmoid fused (CREPE.py:59-75)
  decode      rvc_crepe_decode: fmin/fmax masking, softmax, librosa Viterbi per 512-frame batch
              (as ``predict(batch_size=512)`` decodes per batch), bins -> Hz with the triangular
              dither, periodicity (CREPE.py:85-149)
  smoothing   rvc_crepe_smooth_coarse: mean(f0, 3), median(pd, 3), f0[pd < 0.1] = 0, then the
              pitch shift and coarse mel bins of get_f0

The dither (``scipy.stats.triang.rvs(c=0.5, loc=-20, scale=40)``, CREPE.py:118) is drawn on the host
with numpy's global generator like the reference, or injected through ``dither_fn(T)`` for parity.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib, ops
from .ops import ACT_RELU, ACT_SIGMOID, Conv, check
from .synthetic import CREPE_CAPACITY

HOP = 160
BATCH = 512  # get_f0_crepe's predict(batch_size=512): the Viterbi runs per batch
BN_EPS = 0.0010000000474974513


def _freq_to_bin(f, quantize):
    # CREPE.py:120-121 in torch f32
    return int(quantize(((1200 * torch.log2(torch.tensor(float(f)) / 10)) - 1997.3794084376191) / 20).int())


class CrepeAMD:
    def __init__(self, sd: dict, capacity: str = "full", device: str = "cuda"):
        cin, cout, nfeat = CREPE_CAPACITY[capacity]
        self.capacity, self.device, self.nfeat = capacity, device, nfeat
        self.convs, self.bns = [], []
        for i in range(6):
            w = sd[f"conv{i + 1}.weight"].float()[..., 0]  # [Co][Ci][k]
            self.convs.append(Conv(w, sd[f"conv{i + 1}.bias"].float(), device=device))
            p = f"conv{i + 1}_BN."
            invstd = 1.0 / torch.sqrt(sd[p + "running_var"].float() + BN_EPS)
            alpha = sd[p + "weight"].float() * invstd
            beta = sd[p + "bias"].float() - sd[p + "running_mean"].float() * alpha
            self.bns.append((alpha.to(device), beta.to(device)))
        c6 = cout[5]
        W = sd["classifier.weight"].float()  # [360][h * c6 + c] -> our flatten order [c * 4 + h]
        Wp = W.view(360, nfeat // c6, c6).permute(0, 2, 1).reshape(360, nfeat)
        self.classifier = Conv(Wp.unsqueeze(-1).contiguous(), sd["classifier.bias"].float(), device=device)
        xx, yy = np.meshgrid(range(360), range(360))
        tr = np.maximum(12 - abs(xx - yy), 0)
        tr = tr / tr.sum(axis=1, keepdims=True)
        tiny = np.finfo(np.float64).tiny
        self.log_trans = torch.from_numpy(np.ascontiguousarray(np.log(tr + tiny).T)).to(device)  # [j][k]
        self.log_off = float(np.log(0.0 + tiny))
        self.log_p_init = float(np.log(1.0 / 360 + tiny))
        self.lo, self.hi = _freq_to_bin(50, torch.floor), _freq_to_bin(1100, torch.ceil)
        self.dither_fn = None  # parity hook: dither_fn(T) -> np.ndarray [T] cents

    @classmethod
    def from_file(cls, path, capacity="full", device="cuda"):
        return cls(torch.load(path, map_location="cpu", weights_only=True), capacity, device)

    # ------------------------------------------------------------------ network
    def probabilities(self, audio: torch.Tensor, frame0: int, nb: int, out: torch.Tensor):
        """Sigmoid outputs of frames [frame0, frame0 + nb) into out [360][nb] (a strided view is fine)."""
        lib = _lib.load()
        dev = audio.device
        frames = torch.empty(nb, 1024, device=dev)
        check(lib.rvc_crepe_frames(ops._p(audio), audio.numel(), HOP, frame0, nb, ops._p(frames), ops._stream()),
              "crepe_frames")
        x, L = frames, 1024
        for i in range(6):
            conv = self.convs[i]
            if i == 0:
                Lout = (L + 2 * 254 - 512) // 4 + 1
                y = conv(x, Lout=Lout, stride=4, pad=254, B=nb, Lin=L, x_bstride=L, out_act=ACT_RELU)
            else:
                Lout = L  # pad (31, 32) with k = 64
                y = conv(x, Lout=Lout, pad=31, B=nb, Lin=L, x_bstride=conv.Ci * L, out_act=ACT_RELU)
            Lp = Lout // 2
            alpha, beta = self.bns[i]
            if i < 5:
                h = torch.empty(nb, conv.Co, Lp, device=dev)
                strides = (conv.Co * Lp, Lp, 1)
            else:  # classifier input [c * Lp + h][frame]
                h = torch.empty(conv.Co * Lp, nb, device=dev)
                strides = (1, Lp * nb, nb)
            check(lib.rvc_bn_maxpool(ops._p(y), nb, conv.Co, Lout, ops._p(alpha), ops._p(beta), ops._p(h), *strides,
                                     ops._stream()), "bn_maxpool")
            x, L = h, Lp
        self.classifier(x, out=out, out_act=ACT_SIGMOID)

    # ------------------------------------------------------------------ f0
    def f0_device(self, audio: torch.Tensor, pitch_shift: float = 0.0, trace=None, post=None):
        """audio [N] device f32 (the padded 16 kHz signal) -> (coarse int64 [T], pitchf f32 [T]),
        T = 1 + N // 160."""
        dev = audio.device
        N = audio.numel()
        T = 1 + N // HOP
        probs = torch.empty(360, T, device=dev)
        seq = list(range(0, T, BATCH)) + [T]
        for a, b in zip(seq[:-1], seq[1:]):
            pb = torch.empty(360, b - a, device=dev)
            self.probabilities(audio, a, b - a, pb)
            probs[:, a:b] = pb
        if trace is not None:
            trace["probs"] = probs.t().cpu().numpy().copy()
        if self.dither_fn is not None:
            dither = np.asarray(self.dither_fn(T), dtype=np.float64)
            dither_d = torch.from_numpy(dither.astype(np.float32)).to(dev)
        elif ops.graph_mode():  # captured pass: the same triangular law drawn on the device (graph.py)
            dither_d = ops.rand_triang(torch.empty(T, device=dev), -20.0, 20.0, 0x43524550, 0)
        else:  # scipy.stats.triang.rvs(c=0.5, loc=-20, scale=40): numpy's triangular on [-20, 20]
            dither = np.random.triangular(-20.0, 0.0, 20.0, size=T)
            dither_d = torch.from_numpy(dither.astype(np.float32)).to(dev)
        lib = _lib.load()
        need = lib.rvc_crepe_decode_ws_bytes(T)
        ws = ops._workspace(dev, need, "crepe")
        key = (str(dev), T)  # batch offsets, resident per length (no host copy inside a captured pass)
        seq_off = self.__dict__.setdefault("_seq_off", {}).get(key)
        if seq_off is None:
            seq_off = self._seq_off[key] = torch.tensor(seq, dtype=torch.int64, device=dev)
        f0r = torch.empty(T, device=dev)
        pdr = torch.empty(T, device=dev)
        check(lib.rvc_crepe_decode(ops._p(probs), T, self.lo, self.hi, ops._p(seq_off), len(seq) - 1,
                                   ctypes_ptr(self.log_trans), self.log_off, self.log_p_init, ops._p(dither_d),
                                   ops._p(ws), need, ops._p(f0r), ops._p(pdr), ops._stream()), "crepe_decode")
        coarse = torch.empty(T, dtype=torch.int64, device=dev)
        pitchf = torch.empty(T, device=dev)
        mel_min = 1127 * np.log(1 + 50 / 700)
        mel_max = 1127 * np.log(1 + 1100 / 700)
        check(lib.rvc_crepe_smooth_coarse(ops._p(f0r), ops._p(pdr), T, float(math.pow(2, pitch_shift / 12)),
                                          float(mel_min), float(mel_max), ops._post_ref(post, T), ops._p(coarse),
                                          ops._p(pitchf),
                                          ops._stream()), "crepe_smooth_coarse")
        if trace is not None:
            trace.update(f0_raw=f0r.cpu().numpy(), pd_raw=pdr.cpu().numpy())
        return coarse, pitchf


def ctypes_ptr(t: torch.Tensor):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())
