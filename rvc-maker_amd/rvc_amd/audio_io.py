"""Audio file I/O for the edges of the path (``main/library/utils.py:89-112`` load_audio,
``convert.py:518`` sf.write, ``extract.py:91-100`` read_wave), without soundfile / librosa / soxr
(none is in this image).

* WAV is read and written with ``scipy.io.wavfile``.  Integer PCM is scaled to f32 the way
  libsndfile does for ``dtype=float32`` (x / 2^(bits-1)); multi-channel input is averaged to mono
  (``librosa.to_mono``).  Writing follows soundfile's WAV default subtype, PCM_16.
* Resampling (the reference's ``librosa.resample(res_type="soxr_vhq")``) is a Kaiser-windowed
  polyphase filter (``scipy.signal.resample_poly``).  soxr is absent here, so resampled outputs are
  **parity unpinned**; the 16 kHz input path (no resampling) is the one the parity suite covers.
"""
from __future__ import annotations

import math
import os

import numpy as np
from scipy import signal
from scipy.io import wavfile


def read_wav(path: str) -> tuple[np.ndarray, int]:
    """-> (f32 samples, [n] or [n, channels], sample rate)."""
    sr, x = wavfile.read(path)
    if x.dtype == np.int16:
        y = x.astype(np.float32) / 32768.0
    elif x.dtype == np.int32:
        y = (x.astype(np.float64) / 2147483648.0).astype(np.float32)
    elif x.dtype == np.uint8:
        y = (x.astype(np.float32) - 128.0) / 128.0
    else:
        y = x.astype(np.float32)
    return y, int(sr)


def resample(x: np.ndarray, orig_sr: int, target_sr: int) -> np.ndarray:
    """Band-limited rational resampling (stands in for soxr_vhq; see the module note)."""
    if orig_sr == target_sr:
        return x
    g = math.gcd(int(orig_sr), int(target_sr))
    return signal.resample_poly(x, target_sr // g, orig_sr // g, axis=-1).astype(np.float32)


def load_audio(file: str, sample_rate: int = 16000) -> np.ndarray:
    """utils.py:89-112 without formant shifting: mono f32 at ``sample_rate``, flattened."""
    file = file.strip(" ").strip('"').strip("\n").strip('"').strip(" ")
    if not os.path.isfile(file):
        raise FileNotFoundError(file)
    audio, sr = read_wav(file)
    if audio.ndim > 1:
        audio = audio.mean(axis=1, dtype=np.float32)
    if sr != sample_rate:
        audio = resample(audio, sr, sample_rate)
    return audio.flatten()


def write_wav(path: str, audio: np.ndarray, sr: int) -> None:
    """sf.write(path, audio, sr, format="wav"): PCM_16 (clipped to [-1, 1], scaled by 32767)."""
    pcm = np.round(np.clip(np.asarray(audio, np.float64), -1.0, 1.0) * 32767.0).astype(np.int16)
    wavfile.write(path, int(sr), pcm)
