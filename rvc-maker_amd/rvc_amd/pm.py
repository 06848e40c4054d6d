"""pm f0 on the device: ``VC.get_f0_pm`` (main/inference/convert.py:206-213) -- Praat's To Pitch (ac)
(parselmouth ``Sound.to_pitch_ac(time_step=0.01, voicing_threshold=0.6, pitch_floor=50, pitch_ceiling=1100)``)
and its zero padding to p_len -- followed by get_f0's shift / autotune / f0 file / mel quantiser
(convert.py:304-323), all in csrc/pm.hip (f64 like Praat).

Parity against Praat itself is unpinned: parselmouth is not installed.  The kernels follow the published
algorithm (Boersma 1993, as Praat implements it), restated in oracle/pm.py; tests/test_gpu_pm.py checks the
device against that restatement and both against known pitch tracks.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib, ops

NW = 958  # Praat's nsamp_window for a 50 Hz floor at 16 kHz (3 periods, halved-and-doubled)
BIX = NW // 2


def _p64(t):
    if not t.is_cuda or t.dtype != torch.float64 or not t.is_contiguous():
        raise TypeError(f"rvc_amd pm: expected a contiguous CUDA f64 tensor, got {t.dtype} on {t.device}")
    return ctypes.c_void_p(t.data_ptr())


class PitchPM:
    def __init__(self, device="cuda"):
        # Sound_to_Pitch_any's Hanning window and its normalised autocorrelation, from the library (the same
        # host computation rvc_vc_convert_ex uses)
        w = np.empty(NW, np.float64)
        r = np.empty(BIX + 1, np.float64)
        ops.check(_lib.load().rvc_pm_windows(ctypes.c_void_p(w.ctypes.data), ctypes.c_void_p(r.ctypes.data)),
                  "pm_windows")
        self.window = torch.from_numpy(w).to(device)
        self.window_r = torch.from_numpy(r).to(device)

    def to_pitch_ac(self, x64: torch.Tensor) -> torch.Tensor:
        """x64: device f64 [n] at 16 kHz -> selected frequencies f64 [nframes] (0 = unvoiced)."""
        lib = _lib.load()
        n = x64.numel()
        nf = lib.rvc_pm_frames(n)
        if nf <= 0:
            raise ValueError(f"pm: {n} samples is shorter than one 60 ms analysis window")
        need = lib.rvc_pm_work_bytes(n)
        work = ops._workspace(x64.device, need, "pm")
        f0 = torch.empty(nf, dtype=torch.float64, device=x64.device)
        ops.check(lib.rvc_pm_f0(_p64(x64.contiguous()), n, _p64(self.window), _p64(self.window_r), ops._p(work),
                                need, _p64(f0), ops._stream()), "pm_f0")
        return f0

    def f0_device(self, x64: torch.Tensor, p_len: int, pitch_shift: float = 0.0, post=None):
        """get_f0(..., "pm") on the device: (coarse int64 [max(p_len, nf)], pitchf f32 [same])."""
        f0 = self.to_pitch_ac(x64)
        nf = f0.numel()
        nout = max(p_len, nf)
        coarse = torch.empty(nout, dtype=torch.int64, device=x64.device)
        pitchf = torch.empty(nout, device=x64.device)
        ops.check(_lib.load().rvc_pm_post(_p64(f0), nf, p_len, float(2.0 ** (pitch_shift / 12)),
                                          ops._post_ref(post, nout), ops._p(coarse), ops._p(pitchf), ops._stream()),
                  "pm_post")
        return coarse, pitchf
