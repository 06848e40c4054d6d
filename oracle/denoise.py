"""Oracle: the spectral-gate denoise behind ``convert_audio(clean_audio=True)``.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates
``main/tools/noisereduce.py`` as ``VoiceConverter.convert_audio`` calls it
(``convert.py:514-516``: ``reduce_noise(y, sr, prop_decrease=clean_strength)``, i.e. the
non-stationary gate with every other argument at its default) in numpy float64 -- the
reference runs the whole gate in float64 because ``SpectralGate._read_chunk`` builds each
chunk with ``np.zeros`` (noisereduce.py:76).  Pinned by ``tests/golden/denoise.npz``
(the reference's own ``reduce_noise`` run in the survey container).
"""
from __future__ import annotations

import numpy as np
import torch


def hann_window(n: int) -> np.ndarray:
    """``torch.hann_window(n)`` (periodic, float32 -- noisereduce.py:173) promoted to f64 by stft."""
    return torch.hann_window(n).double().numpy()


def smoothing_filter(sr: float, n_fft: int, hop: int, freq_mask_smooth_hz=500, time_mask_smooth_ms=50):
    """TG._generate_mask_smoothing_filter (noisereduce.py:144-154): a float32 triangle outer product
    (torch.linspace defaults to float32), normalised in float32, used in float64 (:177)."""
    if freq_mask_smooth_hz is None and time_mask_smooth_ms is None:
        return None
    n_gf = 1 if freq_mask_smooth_hz is None else int(freq_mask_smooth_hz / (sr / (n_fft / 2)))
    n_gt = 1 if time_mask_smooth_ms is None else int(time_mask_smooth_ms / ((hop / sr) * 1000))
    if n_gf < 1 or n_gt < 1:
        raise ValueError("mask smoothing window shorter than one bin / frame")
    if n_gf == 1 and n_gt == 1:
        return None

    def tri(n):
        return torch.cat([torch.linspace(0, 1, n + 2)[:-1], torch.linspace(1, 0, n + 2)])[1:-1]

    f = torch.outer(tri(n_gf), tri(n_gt))
    return (f / f.sum()).double().numpy()


def stft(x: np.ndarray, n_fft: int, hop: int, w: np.ndarray) -> np.ndarray:
    """torch.stft(center=True, pad_mode="constant", onesided) -> complex [n_fft//2+1][F]."""
    xp = np.concatenate([np.zeros(n_fft // 2), x, np.zeros(n_fft // 2)])
    F = 1 + len(x) // hop
    idx = np.arange(F)[:, None] * hop + np.arange(n_fft)[None, :]
    return np.fft.rfft(xp[idx] * w[None, :], axis=1).T


def istft(Y: np.ndarray, n_fft: int, hop: int, w: np.ndarray) -> np.ndarray:
    """torch.istft(center=True, length=None): windowed overlap-add / window-square envelope, the
    n_fft//2 centre padding trimmed off both ends -> hop * (F - 1) samples.  With the float32 window
    the reference passes (noisereduce.py:180), torch builds the envelope in float32 (window squared and
    overlap-added in float32, frames in order) -- measured here against torch.istft."""
    F = Y.shape[1]
    fr = np.fft.irfft(Y.T, n=n_fft, axis=1) * w[None, :]
    n = n_fft + hop * (F - 1)
    buf = np.zeros(n)
    env = np.zeros(n, dtype=np.float32)
    w2 = w.astype(np.float32) * w.astype(np.float32)
    for f in range(F):
        buf[f * hop: f * hop + n_fft] += fr[f]
        env[f * hop: f * hop + n_fft] += w2
    env = env.astype(np.float64)
    return buf[n_fft // 2: n - n_fft // 2] / env[n_fft // 2: n - n_fft // 2]


def movemean_same(a: np.ndarray, k: int) -> np.ndarray:
    """conv1d(a, ones(k), padding="same") / k along the last axis (noisereduce.py:164): torch pads
    (k-1)//2 on the left and the rest on the right."""
    left = (k - 1) // 2
    ap = np.concatenate([np.zeros(a.shape[:-1] + (left,)), a, np.zeros(a.shape[:-1] + (k - 1 - left,))], axis=-1)
    c = np.concatenate([np.zeros(a.shape[:-1] + (1,)), np.cumsum(ap, axis=-1)], axis=-1)
    return (c[..., k:] - c[..., :-k]) / k


def conv2d_same(m: np.ndarray, f: np.ndarray) -> np.ndarray:
    """F.conv2d(m, f, padding="same") (cross-correlation, zero padding; odd kernel)."""
    kh, kw = f.shape
    mp = np.pad(m, ((kh // 2, kh // 2), (kw // 2, kw // 2)))
    out = np.zeros_like(m)
    for i in range(kh):
        for j in range(kw):
            out += f[i, j] * mp[i: i + m.shape[0], j: j + m.shape[1]]
    return out


def tg_nonstationary(x: np.ndarray, sr, prop_decrease, n_movemean, n_thresh=2.0, temp_coeff=0.1, n_fft=1024,
                     hop=256, filt=None):
    """TG.forward with nonstationary=True (noisereduce.py:163-180) on one float64 chunk."""
    w = hann_window(n_fft)
    X = stft(x, n_fft, hop, w)
    Xa = np.abs(X)
    Xs = movemean_same(Xa, n_movemean)
    with np.errstate(divide="ignore", invalid="ignore"):
        m = 1.0 / (1.0 + np.exp(-((((Xa - Xs) / Xs) - n_thresh) / temp_coeff)))
    m = prop_decrease * (m * 1.0 - 1.0) + 1.0
    if filt is not None:
        m = conv2d_same(m, filt)
    return istft(X * m, n_fft, hop, w)


def reduce_noise(y, sr, prop_decrease=1.0, time_constant_s=2.0, freq_mask_smooth_hz=500, time_mask_smooth_ms=50,
                 thresh_n_mult_nonstationary=2, sigmoid_slope_nonstationary=10, chunk_size=600000, padding=30000,
                 n_fft=1024, win_length=None, hop_length=None):
    """noisereduce.reduce_noise(stationary=False) (noisereduce.py:199) on a 1-D float32 signal:
    SpectralGate.get_traces chunking (:96-122) around TG (:124-180)."""
    y = np.asarray(y)
    win = n_fft if win_length is None else win_length
    hop = win // 4 if hop_length is None else hop_length
    if win != n_fft:
        raise NotImplementedError("win_length != n_fft")
    n_mm = int(time_constant_s / hop * sr)  # noisereduce.py:193
    filt = smoothing_filter(sr, n_fft, hop, freq_mask_smooth_hz, time_mask_smooth_ms)
    n = y.shape[-1]

    def filt_chunk(s0, e0):  # SpectralGate.filter_chunk (:80-82) through _read_chunk (:73-78)
        i1, i2 = s0 - padding, e0 + padding
        c = np.zeros(i2 - i1)
        a, b = max(i1, 0), min(i2, n)
        c[a - i1: b - i1] = y[a:b]
        return tg_nonstationary(c, sr, prop_decrease, n_mm, float(thresh_n_mult_nonstationary),
                                1.0 / sigmoid_slope_nonstationary, n_fft, hop, filt)[s0 - i1: e0 - i1]

    if chunk_size is not None and n > chunk_size:
        out = np.zeros(n, dtype=y.dtype)
        for ich in range((n - 1) // chunk_size + 1):
            end0 = n - ich * chunk_size if ich == (n - 1) // chunk_size else chunk_size
            out[ich * chunk_size: ich * chunk_size + end0] = filt_chunk(ich * chunk_size, (ich + 1) * chunk_size)[:end0]
        return out
    return filt_chunk(0, n).astype(y.dtype)
