"""Audio edges either side of ``VC.pipeline``: the silence slicer behind
``convert_audio(split_audio=True)`` and dataset preprocessing, the zero-filled re-stitching of the
converted chunks, and the RMS framing they share.

These are host steps in the reference too (numpy over ~100 frames per second of audio, ≈1 ms per
minute of input); they stay on the host here and hand the device path whole chunks.

* ``get_rms``      -- ``main/inference/preprocess.py:119-127`` (same numpy reduction, so the silence
  tests against the threshold see the same f32 values)
* ``Slicer``       -- ``preprocess.py:45-117`` (``slice``: list of chunks)
* ``cut``          -- ``main/library/utils.py:172-237`` (``Slicer2.slice2``: (chunk, start, end) triples)
* ``restore``      -- ``utils.py:239-250``.  Reference quirk kept: ``start``/``end`` and ``total_len``
  are 16 kHz sample positions while the chunks are at the target rate, so the zero gaps are
  16 kHz-sized (``convert.py:510``).

Parity: golden vectors from running the reference's own functions (``tests/golden/edges.npz``,
``tests/golden/make_golden.py gen_edges``).
"""
from __future__ import annotations

import numpy as np


def get_rms(y: np.ndarray, frame_length: int = 2048, hop_length: int = 512) -> np.ndarray:
    """[1][n_frames] frame RMS of y (constant padding of frame_length // 2 each side); frames
    are read as a strided view and reduced along the frame axis, as the reference does."""
    half = int(frame_length // 2)
    yp = np.pad(y, (half, half), mode="constant")
    n = yp.shape[-1] - (frame_length - 1)
    view = np.lib.stride_tricks.as_strided(yp, shape=(n, frame_length), strides=(yp.strides[-1], yp.strides[-1]))
    frames = np.moveaxis(view, -1, -2)[:, ::hop_length]  # [frame_length][n_frames]
    return np.sqrt(np.mean(np.abs(frames) ** 2, axis=-2, keepdims=True))


class Slicer:
    """Silence slicer: threshold in dB, lengths in ms; internally in hops of ``hop_size`` ms."""

    def __init__(self, sr, threshold=-40.0, min_length=5000, min_interval=300, hop_size=20, max_sil_kept=5000):
        if not min_length >= min_interval >= hop_size:
            raise ValueError("min_length >= min_interval >= hop_size is required")
        if not max_sil_kept >= hop_size:
            raise ValueError("max_sil_kept >= hop_size is required")
        interval = sr * min_interval / 1000
        self.threshold = 10 ** (threshold / 20.0)
        self.hop_size = round(sr * hop_size / 1000)
        self.win_size = min(round(interval), 4 * self.hop_size)
        self.min_length = round(sr * min_length / 1000 / self.hop_size)
        self.min_interval = round(interval / self.hop_size)
        self.max_sil_kept = round(sr * max_sil_kept / 1000 / self.hop_size)

    def _apply_slice(self, waveform, begin, end):
        a = begin * self.hop_size
        if waveform.ndim > 1:
            return waveform[:, a: min(waveform.shape[1], end * self.hop_size)]
        return waveform[a: min(waveform.shape[0], end * self.hop_size)]

    def silence_tags(self, rms_list: np.ndarray) -> list[tuple[int, int]]:
        """(begin, end) hop indices of the silences to cut, by the reference's state machine."""
        tags = []
        sil, clip = None, 0
        keep = self.max_sil_kept
        for i, r in enumerate(rms_list):
            if r < self.threshold:
                if sil is None:
                    sil = i
                continue
            if sil is None:
                continue
            leading = sil == 0 and i > keep
            middle = i - sil >= self.min_interval and i - clip >= self.min_length
            if not leading and not middle:
                sil = None
                continue
            if i - sil <= keep:  # short silence: cut at its quietest hop
                pos = int(rms_list[sil: i + 1].argmin()) + sil
                tags.append((0, pos) if sil == 0 else (pos, pos))
                clip = pos
            elif i - sil <= 2 * keep:  # medium: keep up to max_sil_kept on each side
                pos = int(rms_list[i - keep: sil + keep + 1].argmin()) + i - keep
                pos_r = int(rms_list[i - keep: i + 1].argmin()) + i - keep
                if sil == 0:
                    tags.append((0, pos_r))
                    clip = pos_r
                else:
                    pos_l = int(rms_list[sil: sil + keep + 1].argmin()) + sil
                    tags.append((min(pos_l, pos), max(pos_r, pos)))
                    clip = max(pos_r, pos)
            else:  # long: quietest hop near each edge
                pos_r = int(rms_list[i - keep: i + 1].argmin()) + i - keep
                if sil == 0:
                    tags.append((0, pos_r))
                else:
                    tags.append((int(rms_list[sil: sil + keep + 1].argmin()) + sil, pos_r))
                clip = pos_r
            sil = None
        total = rms_list.shape[0]
        if sil is not None and total - sil >= self.min_interval:  # trailing silence
            tags.append((int(rms_list[sil: min(total, sil + keep) + 1].argmin()) + sil, total + 1))
        return tags

    def _rms(self, samples):
        return get_rms(samples, self.win_size, self.hop_size).squeeze(0)

    def slice(self, waveform: np.ndarray) -> list[np.ndarray]:
        """preprocess.py:63-117: the non-silent chunks."""
        samples = waveform.mean(axis=0) if waveform.ndim > 1 else waveform
        if samples.shape[0] <= self.min_length:
            return [waveform]
        rms_list = self._rms(samples)
        tags = self.silence_tags(rms_list)
        if not tags:
            return [waveform]
        total = rms_list.shape[0]
        chunks = []
        if tags[0][0] > 0:
            chunks.append(self._apply_slice(waveform, 0, tags[0][0]))
        for a, b in zip(tags[:-1], tags[1:]):
            chunks.append(self._apply_slice(waveform, a[1], b[0]))
        if tags[-1][1] < total:
            chunks.append(self._apply_slice(waveform, tags[-1][1], total))
        return chunks

    def slice2(self, waveform: np.ndarray) -> list[tuple[np.ndarray, int, int]]:
        """utils.py:176-234: (chunk, start sample, end sample) triples."""
        samples = waveform.mean(axis=0) if waveform.ndim > 1 else waveform
        if samples.shape[0] <= self.min_length:
            return [(waveform, 0, samples.shape[0])]
        rms_list = self._rms(samples)
        tags = self.silence_tags(rms_list)
        if not tags:
            return [(waveform, 0, samples.shape[-1])]
        h = self.hop_size
        total = rms_list.shape[0]
        chunks = []
        if tags[0][0] > 0:
            chunks.append((self._apply_slice(waveform, 0, tags[0][0]), 0, tags[0][0] * h))
        for a, b in zip(tags[:-1], tags[1:]):
            chunks.append((self._apply_slice(waveform, a[1], b[0]), a[1] * h, b[0] * h))
        if tags[-1][1] < total:
            chunks.append((self._apply_slice(waveform, tags[-1][1], total), tags[-1][1] * h, samples.shape[-1]))
        return chunks


def cut(audio: np.ndarray, sr: int, db_thresh: float = -60, min_interval: int = 250):
    """utils.py:172-237 (``convert_audio(split_audio=True)`` calls it with -60 dB, 500 ms)."""
    return Slicer(sr=sr, threshold=db_thresh, min_interval=min_interval).slice2(audio)


def restore(segments, total_len: int, dtype=np.float32) -> np.ndarray:
    """utils.py:239-250: concatenate (start, end, chunk) with zero gaps; see the module note."""
    out, last = [], 0
    for start, end, seg in segments:
        if start > last:
            out.append(np.zeros(start - last, dtype=dtype))
        out.append(seg)
        last = end
    if last < total_len:
        out.append(np.zeros(total_len - last, dtype=dtype))
    return np.concatenate(out, axis=-1)
