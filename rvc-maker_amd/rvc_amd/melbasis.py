"""Mel filterbank for RMVPE's MelSpectrogram (``RMVPE.py:151``).

The reference calls ``librosa.filters.mel(sr=16000, n_fft=1024, n_mels=128,
fmin=30, fmax=8000, htk=True)`` (Slaney area normalisation, float32 output).
librosa is not installed in this image, so this is a restatement of its
published algorithm (librosa 0.10 ``filters.mel`` / ``mel_frequencies`` /
``hz_to_mel(htk=True)``): triangular filters between consecutive mel points,
f64 arithmetic, cast to float32 on store.  Parity vs librosa itself is
UNPINNED (no librosa output exists in the reference tree); everything
downstream of the basis is pinned by the golden vectors, which were generated
with this same basis standing in for librosa.
"""
from __future__ import annotations

import numpy as np


def hz_to_mel_htk(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, dtype=np.float64) / 700.0)


def mel_to_hz_htk(m):
    return 700.0 * (10.0 ** (np.asarray(m, dtype=np.float64) / 2595.0) - 1.0)


def mel_filterbank(sr=16000, n_fft=1024, n_mels=128, fmin=30.0, fmax=8000.0) -> np.ndarray:
    n_bins = 1 + n_fft // 2
    weights = np.zeros((n_mels, n_bins), dtype=np.float32)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = mel_to_hz_htk(np.linspace(hz_to_mel_htk(fmin), hz_to_mel_htk(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights
