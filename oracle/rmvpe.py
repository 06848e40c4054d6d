"""Oracle: RMVPE f0 (mel -> DeepUnet -> BiGRU -> salience -> decode) on torch-CPU.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates
``main/library/predictors/RMVPE.py``.  The mel basis comes from
``rvc_amd.melbasis`` (a restatement of ``librosa.filters.mel``: librosa is not
installed, so the basis is parity-unpinned against librosa >= 0.10.2; the
golden vectors pin everything downstream of it).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

N_MELS, N_CLASS = 128, 360


def load_weights(sd: dict, dtype=torch.float32) -> dict:
    """Float tensors of the state dict in ``dtype`` (f32 = the reference's arithmetic; f64 is the
    diagnostic "exact" run the parity tests measure both the reference's and the device's f32 noise against)."""
    return {k: v.to(dtype) for k, v in sd.items() if v.is_floating_point()}


def mel_spectrogram(audio, mel_basis, n_fft=1024, hop=160, clamp=1e-5):
    """MelSpectrogram.forward, keyshift 0, center=True (RMVPE.py:162-181)."""
    win = torch.hann_window(n_fft).to(audio.dtype)  # the f32 window (RMVPE.py:166), upcast in an f64 run
    fft = torch.stft(audio, n_fft=n_fft, hop_length=hop, win_length=n_fft, window=win, center=True,
                     return_complex=True)
    mag = torch.sqrt(fft.real.pow(2) + fft.imag.pow(2))
    mel = torch.matmul(mel_basis.to(mag.dtype), mag)
    return torch.log(torch.clamp(mel, min=clamp))


def _bn(W, p, x):
    return F.batch_norm(x, W[p + ".running_mean"], W[p + ".running_var"], W[p + ".weight"], W[p + ".bias"],
                        False, 0.0, 1e-5)


def _cbr(W, p, x):
    """ConvBlockRes.forward (RMVPE.py:21-22)."""
    h = F.conv2d(x, W[p + ".conv.0.weight"], None, 1, 1)
    h = F.relu(_bn(W, p + ".conv.1", h))
    h = F.conv2d(h, W[p + ".conv.3.weight"], None, 1, 1)
    h = F.relu(_bn(W, p + ".conv.4", h))
    if (p + ".shortcut.weight") in W:
        return h + F.conv2d(x, W[p + ".shortcut.weight"], W[p + ".shortcut.bias"])
    return h + x


def unet(W, x, n_blocks=4):
    """DeepUnet.forward (RMVPE.py:132-134) incl. Encoder/Intermediate/Decoder."""
    x = _bn(W, "unet.encoder.bn", x)
    skips = []
    for l in range(5):
        for b in range(n_blocks):
            x = _cbr(W, f"unet.encoder.layers.{l}.conv.{b}", x)
        skips.append(x)
        x = F.avg_pool2d(x, 2)
    for l in range(4):
        for b in range(n_blocks):
            x = _cbr(W, f"unet.intermediate.layers.{l}.conv.{b}", x)
    for l in range(5):
        p = f"unet.decoder.layers.{l}"
        x = F.conv_transpose2d(x, W[p + ".conv1.0.weight"], None, (2, 2), (1, 1), (1, 1))
        x = F.relu(_bn(W, p + ".conv1.1", x))
        x = torch.cat((x, skips[-1 - l]), dim=1)
        for b in range(n_blocks):
            x = _cbr(W, f"{p}.conv2.{b}", x)
    return x


def _gru_dir(x, w_ih, w_hh, b_ih, b_hh, reverse):
    """One direction of nn.GRU (r, z, n gate order)."""
    T = x.shape[0]
    H = w_hh.shape[1]
    gi = F.linear(x, w_ih, b_ih)
    h = torch.zeros(H, dtype=x.dtype)
    out = torch.empty(T, H, dtype=x.dtype)
    steps = range(T - 1, -1, -1) if reverse else range(T)
    for t in steps:
        gh = F.linear(h, w_hh, b_hh)
        r = torch.sigmoid(gi[t, :H] + gh[:H])
        z = torch.sigmoid(gi[t, H:2 * H] + gh[H:2 * H])
        n = torch.tanh(gi[t, 2 * H:] + r * gh[2 * H:])
        h = (h - n) * z + n
        out[t] = h
    return out


def bigru(W, x):
    """BiGRU (RMVPE.py:254-260) on [1, T, 384] -> [1, T, 512]."""
    p = "fc.0.gru."
    f = _gru_dir(x[0], W[p + "weight_ih_l0"], W[p + "weight_hh_l0"], W[p + "bias_ih_l0"], W[p + "bias_hh_l0"], False)
    b = _gru_dir(x[0], W[p + "weight_ih_l0_reverse"], W[p + "weight_hh_l0_reverse"], W[p + "bias_ih_l0_reverse"],
                 W[p + "bias_hh_l0_reverse"], True)
    return torch.cat([f, b], dim=-1).unsqueeze(0)


def bigru_torch(W, x):
    """Same as ``bigru`` through torch's own GRU kernel (what the reference executes)."""
    gru = torch.nn.GRU(384, 256, num_layers=1, batch_first=True, bidirectional=True).to(x.dtype)
    gru.load_state_dict({k[len("fc.0.gru."):]: W[k] for k in W if k.startswith("fc.0.gru.")})
    with torch.no_grad():
        return gru(x)[0]


def e2e(W, mel):
    """E2E.forward (RMVPE.py:143-144): mel [1, 128, T] -> salience [1, T, 360]."""
    x = unet(W, mel.transpose(-1, -2).unsqueeze(1))
    x = F.conv2d(x, W["cnn.weight"], W["cnn.bias"], 1, 1)
    x = x.transpose(1, 2).flatten(-2)
    x = bigru_torch(W, x)
    return torch.sigmoid(F.linear(x, W["fc.1.weight"], W["fc.1.bias"]))


def mel2hidden(W, mel):
    """RMVPE.mel2hidden (RMVPE.py:210-215): reflect-pad frames to a multiple of 32."""
    n = mel.shape[-1]
    mel = F.pad(mel, (0, 32 * ((n - 1) // 32 + 1) - n), mode="reflect")
    return e2e(W, mel)[:, :n]


CENTS_MAPPING = np.pad(20 * np.arange(N_CLASS) + 1997.3794084376191, (4, 4))  # RMVPE.py:207-208


def to_local_average_cents(salience, thred=0.05):
    """RMVPE.py:236-252 (vectorised; same arithmetic order per frame)."""
    center = np.argmax(salience, axis=1)
    sal = np.pad(salience, ((0, 0), (4, 4)))
    center += 4
    idx = center[:, None] + np.arange(-4, 5)[None, :]
    todo_sal = np.take_along_axis(sal, idx, axis=1)
    todo_cents = CENTS_MAPPING[idx]
    devided = np.sum(todo_sal * todo_cents, 1) / np.sum(todo_sal, 1)
    devided[np.max(sal, axis=1) <= thred] = 0
    return devided


def decode(salience, thred=0.03):
    """RMVPE.decode (RMVPE.py:217-221)."""
    f0 = 10 * (2 ** (to_local_average_cents(salience, thred=thred) / 1200))
    f0[f0 == 10] = 0
    return f0


def infer_from_audio(W, mel_basis, audio: np.ndarray, thred=0.03) -> np.ndarray:
    """RMVPE.infer_from_audio (RMVPE.py:223-226): f64 audio [N] -> f64 f0 [1 + N//160]."""
    mel = mel_spectrogram(torch.from_numpy(audio).float().unsqueeze(0), mel_basis)
    hidden = mel2hidden(W, mel)
    return decode(hidden.squeeze(0).numpy(), thred=thred)
