"""Spectral-gate denoise on the device: drop-in for ``main/tools/noisereduce.py:reduce_noise``.

``VoiceConverter.convert_audio`` runs it on the converted waveform when ``clean_audio`` is set
(``convert.py:514-516``: ``reduce_noise(y=audio_output, sr=target_sr, prop_decrease=clean_strength)``),
which is the non-stationary gate (``TG``, noisereduce.py:124-180) over ``SpectralGate.get_traces``'
chunks (:96-122).  The whole gate runs in f64 in ``csrc/denoise.hip`` (the reference computes in
float64: ``_read_chunk`` builds each chunk with ``np.zeros``, :76); the host only computes the two
constants the reference builds with torch on its CPU -- the float32 Hann window (:173) and the
float32 mask-smoothing triangle (:144-154).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check


def smoothing_filter(sr, n_fft, hop, freq_mask_smooth_hz=500, time_mask_smooth_ms=50):
    """TG._generate_mask_smoothing_filter (noisereduce.py:144-154) -> f64 [2nf+1][2nt+1] or None."""
    if freq_mask_smooth_hz is None and time_mask_smooth_ms is None:
        return None
    n_gf = 1 if freq_mask_smooth_hz is None else int(freq_mask_smooth_hz / (sr / (n_fft / 2)))
    if n_gf < 1:
        raise ValueError(f"freq_mask_smooth_hz must be at least {int(sr / (n_fft / 2))} Hz")
    n_gt = 1 if time_mask_smooth_ms is None else int(time_mask_smooth_ms / ((hop / sr) * 1000))
    if n_gt < 1:
        raise ValueError(f"time_mask_smooth_ms must be at least {int((hop / sr) * 1000)} ms")
    if n_gf == 1 and n_gt == 1:
        return None

    def tri(n):  # cat([linspace(0, 1, n + 1, endpoint=False), linspace(1, 0, n + 2)])[1:-1], float32
        return torch.cat([torch.linspace(0, 1, n + 2)[:-1], torch.linspace(1, 0, n + 2)])[1:-1]

    f = torch.outer(tri(n_gf), tri(n_gt))
    return (f / f.sum()).double()


class SpectralGateAMD:
    """The gate's constants on the device, for one (sr, parameters) combination."""

    def __init__(self, sr, prop_decrease=1.0, time_constant_s=2.0, freq_mask_smooth_hz=500, time_mask_smooth_ms=50,
                 thresh_n_mult_nonstationary=2, sigmoid_slope_nonstationary=10, chunk_size=600000, padding=30000,
                 n_fft=1024, win_length=None, hop_length=None, device="cuda"):
        if not 0.0 <= prop_decrease <= 1.0:
            raise ValueError("prop_decrease must be in [0, 1]")  # noisereduce.py:130
        win = n_fft if win_length is None else win_length
        if win != n_fft:
            raise NotImplementedError("win_length != n_fft")
        self.hop = win // 4 if hop_length is None else hop_length
        self.n_fft = n_fft
        self.win = torch.hann_window(win).double().to(device)
        f = smoothing_filter(sr, n_fft, self.hop, freq_mask_smooth_hz, time_mask_smooth_ms)
        self.filt = f.contiguous().to(device) if f is not None else None
        a = _lib.DenoiseArgs()
        a.chunk_size = chunk_size if chunk_size is not None else 0
        a.padding = padding
        a.n_fft, a.hop = n_fft, self.hop
        a.n_movemean = int(time_constant_s / self.hop * sr)  # noisereduce.py:193
        a.filt_h, a.filt_w = (self.filt.shape if self.filt is not None else (0, 0))
        a.prop_decrease = float(prop_decrease)
        a.n_thresh = float(thresh_n_mult_nonstationary)
        a.temp_coeff = 1.0 / sigmoid_slope_nonstationary
        a.window = ctypes.c_void_p(self.win.data_ptr())
        a.filt = ctypes.c_void_p(self.filt.data_ptr()) if self.filt is not None else None
        self.args = a

    def __call__(self, y: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """y: device f32 [n] -> gated f32 [n] (stream-ordered on the current stream)."""
        if y.dtype != torch.float32 or not y.is_cuda or y.dim() != 1:
            raise TypeError("denoise: expected a 1-D CUDA float32 tensor")
        y = y.contiguous()
        n = y.numel()
        lib = _lib.load()
        need = lib.rvc_denoise_work_bytes(n, ctypes.byref(self.args))
        if need < 0:
            raise ValueError(f"denoise: {lib.rvc_last_error().decode()}")
        work = torch.empty((need + 7) // 8, dtype=torch.float64, device=y.device)
        if out is None:
            out = torch.empty_like(y)
        stream = ctypes.c_void_p(torch.cuda.current_stream(y.device).cuda_stream)
        check(lib.rvc_denoise(ctypes.c_void_p(y.data_ptr()), n, ctypes.byref(self.args),
                              ctypes.c_void_p(work.data_ptr()), work.numel() * 8, ctypes.c_void_p(out.data_ptr()),
                              stream), "denoise")
        return out


def reduce_noise(y, sr, stationary=False, y_noise=None, prop_decrease=1.0, time_constant_s=2.0,
                 freq_mask_smooth_hz=500, time_mask_smooth_ms=50, thresh_n_mult_nonstationary=2,
                 sigmoid_slope_nonstationary=10, tmp_folder=None, chunk_size=600000, padding=30000, n_fft=1024,
                 win_length=None, hop_length=None, clip_noise_stationary=True, use_tqdm=False, device="cuda"):
    """noisereduce.reduce_noise (noisereduce.py:199) on the device.  ``y``: 1-D numpy array or device
    tensor; returns the same kind (numpy in the input's dtype, like the reference).  The stationary gate
    is not on the convert_audio path and raises."""
    if stationary or y_noise is not None:
        raise NotImplementedError("stationary gating is not on the convert_audio path (convert.py:516)")
    gate = SpectralGateAMD(sr, prop_decrease, time_constant_s, freq_mask_smooth_hz, time_mask_smooth_ms,
                           thresh_n_mult_nonstationary, sigmoid_slope_nonstationary, chunk_size, padding, n_fft,
                           win_length, hop_length, device=device)
    if torch.is_tensor(y):
        return gate(y.float())
    arr = np.asarray(y)
    if arr.ndim != 1:
        raise ValueError("denoise: mono signals only (convert_audio passes a 1-D waveform)")
    out = gate(torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32)).to(device))
    return out.cpu().numpy().astype(arr.dtype)
