"""Oracle: ``VC.pipeline`` (main/inference/convert.py:388-458) on torch-CPU / numpy / scipy.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  f0 method "rmvpe" or crepe, optional
IVF-Flat retrieval through oracle.ivf (faiss itself is absent: parity unpinned), f0
autotune, f0 file and volume envelope (change_rms; its librosa RMS is restated, parity
unpinned vs librosa).  Noise is injected through ``noise(seg, name, shape)``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F
from scipy import signal

from . import contentvec as cv
from . import rmvpe as rm
from . import synth as sy

BH, AH = signal.butter(N=5, Wn=48, btype="high", fs=16000)  # convert.py:30


class Consts:
    """VC.__init__ (convert.py:181-204) with the fp32 Config windows (1, 6, 38, 41)."""

    def __init__(self, tgt_sr, x_pad=1, x_query=6, x_center=38, x_max=41):
        self.sr, self.window = 16000, 160
        self.x_pad = x_pad
        self.t_pad = self.sr * x_pad
        self.t_pad_tgt = tgt_sr * x_pad
        self.t_pad2 = self.t_pad * 2
        self.t_query = self.sr * x_query
        self.t_center = self.sr * x_center
        self.t_max = self.sr * x_max
        self.f0_min, self.f0_max = 50, 1100
        self.f0_mel_min = 1127 * np.log(1 + self.f0_min / 700)
        self.f0_mel_max = 1127 * np.log(1 + self.f0_max / 700)


REF_NOTES = [49.00, 51.91, 55.00, 58.27, 61.74, 65.41, 69.30, 73.42, 77.78, 82.41, 87.31, 92.50, 98.00, 103.83,
             110.00, 116.54, 123.47, 130.81, 138.59, 146.83, 155.56, 164.81, 174.61, 185.00, 196.00, 207.65, 220.00,
             233.08, 246.94, 261.63, 277.18, 293.66, 311.13, 329.63, 349.23, 369.99, 392.00, 415.30, 440.00, 466.16,
             493.88, 523.25, 554.37, 587.33, 622.25, 659.25, 698.46, 739.99, 783.99, 830.61, 880.00, 932.33, 987.77,
             1046.50]  # VC.__init__ ref_freqs (convert.py:198)


def autotune_f0(f0: np.ndarray, strength: float) -> np.ndarray:
    """Autotune.autotune_f0 (convert.py:172-179): each frame moves toward the nearest reference note
    (first on ties), unvoiced frames included; arithmetic in the array's dtype (NumPy 2)."""
    out = np.zeros_like(f0)
    for i, freq in enumerate(f0):
        out[i] = freq + (min(REF_NOTES, key=lambda x: abs(x - freq)) - freq) * strength
    return out


def f0_override(inp_f0: np.ndarray, x_pad: int, tf0: int = 100):
    """convert.py:316-318: (np.interp of the f0 file at 100 frames/s, first frame index)."""
    n = np.round((inp_f0[:, 0].max() - inp_f0[:, 0].min()) * tf0 + 1).astype(np.int16)
    return np.interp(list(range(n)), inp_f0[:, 0] * 100, inp_f0[:, 1]), x_pad * tf0


def rms_librosa(y: np.ndarray, frame_length: int, hop_length: int) -> np.ndarray:
    """librosa.feature.rms(y=y, frame_length, hop_length) of librosa >= 0.10 (center=True,
    pad_mode="constant", dtype=float32 squares) -> [1, 1 + len(y) // hop_length].  librosa is absent
    here: this restatement is PARITY UNPINNED against librosa itself."""
    yp = np.pad(y, (frame_length // 2, frame_length // 2), mode="constant")
    n = 1 + (yp.shape[0] - frame_length) // hop_length
    frames = np.lib.stride_tricks.as_strided(yp, shape=(frame_length, n),
                                             strides=(yp.strides[0], hop_length * yp.strides[0]))
    power = np.mean(np.power(frames, 2, dtype=np.float32), axis=-2, keepdims=True)
    return np.sqrt(power)


def change_rms(source_audio, source_rate, target_audio, target_rate, rate):
    """change_rms (convert.py:150-152): torch linear interpolation of both RMS envelopes to the output
    length, gain = rms1^(1-rate) * max(rms2, 1e-6)^(rate-1)."""
    n = target_audio.shape[0]
    r2 = F.interpolate(torch.from_numpy(rms_librosa(target_audio, target_rate // 2 * 2, target_rate // 2)).float()
                       .unsqueeze(0), size=n, mode="linear").squeeze()
    r1 = F.interpolate(torch.from_numpy(rms_librosa(source_audio, source_rate // 2 * 2, source_rate // 2)).float()
                       .unsqueeze(0), size=n, mode="linear").squeeze()
    return (target_audio * (torch.pow(r1, 1 - rate) * torch.pow(torch.maximum(r2, torch.zeros_like(r2) + 1e-6),
                                                               rate - 1)).numpy())


def coarse_f0(f0: np.ndarray, pitch: float, c: Consts, autotune_strength=None, inp_f0=None):
    """VC.get_f0 tail (convert.py:311-323): optional autotune, shift, optional f0-file override, quantiser."""
    if autotune_strength is not None:
        f0 = autotune_f0(f0, autotune_strength)
    f0 = f0 * pow(2, pitch / 12)
    if inp_f0 is not None:
        rep, a = f0_override(inp_f0, c.x_pad)
        f0[a: a + len(rep)] = rep[:f0[a: a + len(rep)].shape[0]]
    f0_mel = 1127 * np.log(1 + f0 / 700)
    f0_mel[f0_mel > 0] = (f0_mel[f0_mel > 0] - c.f0_mel_min) * 254 / (c.f0_mel_max - c.f0_mel_min) + 1
    f0_mel[f0_mel <= 1] = 1
    f0_mel[f0_mel > 255] = 255
    return np.rint(f0_mel).astype(np.int32), f0.copy()


def segment_points(audio: np.ndarray, c: Consts):
    """Quiet-point segmentation for long inputs (convert.py:404-412)."""
    opt_ts = []
    audio_pad = np.pad(audio, (c.window // 2, c.window // 2), mode="reflect")
    if audio_pad.shape[0] > c.t_max:
        audio_sum = np.zeros_like(audio)
        for i in range(c.window):
            audio_sum += audio_pad[i: i - c.window]
        for t in range(c.t_center, audio.shape[0], c.t_center):
            seg = np.abs(audio_sum[t - c.t_query: t + c.t_query])
            opt_ts.append(t - c.t_query + np.where(seg == seg.min())[0][0])
    return opt_ts


def voice_conversion(Wc, Ws, cfg, sid, audio0, pitch, pitchf, version, protect, z_noise, sine_noise, trace=None,
                     index=None, big_npy=None, index_rate=0.0, embed_suffix=".pt"):
    """VC.voice_conversion (convert.py:328-386), ``.pth`` model; the embedder is ``.pt`` (fairseq
    extract_features at layer 9 (v1) / 12 (v2), convert.py:337-340) or ``.safetensors`` (transformers
    ``model(feats)["last_hidden_state"]``: every layer, final_proj on it for v1, convert.py:342-345) -- the same
    network (``Wc`` in fairseq names); ``index`` is an ``IVFFlatIndex`` searched by the numpy restatement in
    ``oracle.ivf`` (convert.py:349-359)."""
    window = 160
    feats = torch.from_numpy(audio0).float().view(1, -1)
    with torch.no_grad():
        if embed_suffix == ".safetensors":
            x = cv.extract_features(Wc, feats, cv.n_layers(Wc))
        else:
            x = cv.extract_features(Wc, feats, 9 if version == "v1" else 12)
        feats = cv.final_proj(Wc, x) if version == "v1" else x
        if trace is not None:
            trace["feats"] = feats.clone()
        if protect < 0.5:
            feats0 = feats.clone()
        if index is not None and big_npy is not None and index_rate != 0:
            from . import ivf
            npy = feats[0].cpu().numpy()
            D, I = ivf.search(index, npy, k=8)
            feats = torch.from_numpy(ivf.blend(npy, D, I, big_npy, index_rate)).unsqueeze(0)
            if trace is not None:
                trace.update(ivf_D=D, ivf_I=I)
        feats = F.interpolate(feats.permute(0, 2, 1), scale_factor=2).permute(0, 2, 1)
        if protect < 0.5:
            feats0 = F.interpolate(feats0.permute(0, 2, 1), scale_factor=2).permute(0, 2, 1)
        p_len = audio0.shape[0] // window
        if feats.shape[1] < p_len:
            p_len = feats.shape[1]
            pitch = pitch[:, :p_len]
            pitchf = pitchf[:, :p_len]
        if protect < 0.5:
            pitchff = pitchf.clone()
            pitchff[pitchf > 0] = 1
            pitchff[pitchf < 1] = protect
            pitchff = pitchff.unsqueeze(-1)
            feats = (feats * pitchff + feats0 * (1 - pitchff)).to(feats0.dtype)
        p_len_t = torch.tensor([p_len]).long()
        o, _, (z, z_p, m_p, logs_p) = sy.infer(Ws, cfg, feats.float(), p_len_t, pitch, pitchf.float(), sid,
                                               z_noise, sine_noise)
        if trace is not None:
            trace.update(phone=feats, z_p=z_p, z=z, m_p=m_p, logs_p=logs_p)
    return o[0, 0].numpy()


def pipeline(Wc, Ws, Wr, mel_basis, cfg, sid, audio, pitch, version, protect, noise, trace=None, index=None,
             index_rate=0.0, crepe=None, autotune_strength=None, inp_f0=None, volume_envelope=1.0, f0_track=None,
             pm=False, embed_suffix=".pt"):
    """VC.pipeline (convert.py:388-458): f0 = rmvpe (or crepe), optional index, autotune, f0 file
    (``inp_f0`` [n][2] f32) and volume envelope.

    noise(seg_index, name, shape) -> torch tensor for "z" [1, 192, T] and "sine" [1, T*upp, 1].
    ``f0_track`` (f64 [1 + len(padded) // 160]) replaces the f0 estimator's raw output: the parity tests
    use it to check everything after the f0 decision against the device's own decisions."""
    tgt_sr = cfg[-1]
    upp = int(np.prod(cfg[12]))
    c = Consts(tgt_sr)
    audio = signal.filtfilt(BH, AH, audio)
    opt_ts = segment_points(audio, c)
    s = 0
    t = None
    audio_opt = []
    audio_pad = np.pad(audio, (c.t_pad, c.t_pad), mode="reflect")
    sid_t = torch.tensor(sid).unsqueeze(0).long()
    big_npy = index.reconstruct_n(0, index.ntotal) if index is not None and index_rate != 0 else None
    p_len = audio_pad.shape[0] // c.window
    if f0_track is not None:
        f0 = np.array(f0_track, dtype=np.float64, copy=True)
        if f0.shape != (1 + audio_pad.shape[0] // c.window,):
            raise ValueError(f"f0_track has {f0.shape}, expected {(1 + audio_pad.shape[0] // c.window,)}")
    elif pm:  # f0_method "pm": get_f0_pm (convert.py:206-213), restated in oracle/pm.py (parity unpinned)
        from . import pm as opm
        f0 = opm.get_f0_pm(audio_pad, p_len)
    elif crepe is not None:  # f0_method "crepe-<capacity>": (state dict, capacity, dither cents [T])
        from . import crepe as oc
        csd, capacity, dither = crepe
        f0 = oc.get_f0_crepe(csd, audio_pad, dither, capacity)
    else:
        f0 = rm.infer_from_audio(Wr, mel_basis, audio_pad, thred=0.03)
    pitch_c, pitchf = coarse_f0(f0, pitch, c, autotune_strength, inp_f0)
    if trace is not None:
        trace["f0_raw"] = f0
        trace["coarse"] = pitch_c.copy()
    pitch_c, pitchf = pitch_c[:p_len], pitchf[:p_len]
    pitch_t = torch.tensor(pitch_c).unsqueeze(0).long()
    pitchf_t = torch.tensor(pitchf).unsqueeze(0).float()

    def run(seg, a0, pch, pchf):
        T = min(a0.shape[0] // c.window, 2 * cv.frames(a0.shape[0]))
        tr = {} if trace is not None else None
        out = voice_conversion(Wc, Ws, cfg, sid_t, a0, pch, pchf, version, protect,
                               noise(seg, "z", (1, cfg[2], T)), noise(seg, "sine", (1, T * upp, 1)), tr,
                               index=index, big_npy=big_npy, index_rate=index_rate, embed_suffix=embed_suffix)
        if trace is not None:
            trace.setdefault("segments", []).append(tr)
        return out[c.t_pad_tgt: -c.t_pad_tgt]

    seg = 0
    for t in opt_ts:
        t = t // c.window * c.window
        audio_opt.append(run(seg, audio_pad[s: t + c.t_pad2 + c.window],
                             pitch_t[:, s // c.window: (t + c.t_pad2) // c.window],
                             pitchf_t[:, s // c.window: (t + c.t_pad2) // c.window]))
        s = t
        seg += 1
    audio_opt.append(run(seg, audio_pad[t:] if t is not None else audio_pad,
                         pitch_t[:, t // c.window:] if t is not None else pitch_t,
                         pitchf_t[:, t // c.window:] if t is not None else pitchf_t))
    audio_opt = np.concatenate(audio_opt)
    if volume_envelope != 1:
        audio_opt = change_rms(audio, c.sr, audio_opt, c.sr, volume_envelope)
    audio_max = np.abs(audio_opt).max() / 0.99
    if audio_max > 1:
        audio_opt /= audio_max
    return audio_opt
