"""TEST INFRASTRUCTURE ONLY (parity oracle; never imported by the product path).

CREPE f0 (``VC.get_f0_crepe``, convert.py:230-237 -> main/library/predictors/CREPE.py) restated on
torch-CPU / numpy:

* ``preprocess``   CREPE.py:151-171: frames of 1024 at hop 160, zero-padded by 512 each side, each
                   frame made zero-mean and divided by max(1e-10, unbiased std)
* ``network``      CREPE.py:11-75: 6 x [pad, Conv(k x 1), ReLU, BatchNorm (eps 1e-3), MaxPool(2 x 1)],
                   then Linear(in_features, 360) + sigmoid over the (position, channel)-ordered flatten
* ``postprocess``  CREPE.py:141-149: bins < floor-bin(fmin) and >= ceil-bin(fmax) set to -inf,
                   softmax over bins, ``librosa.sequence.viterbi`` with the CREPE transition
                   (max(12 - |i - j|, 0), row-normalised), bins -> Hz with a triangular dither
                   (scipy.stats.triang c=0.5 on [-20, 20] cents; injected here), periodicity
* ``mean`` / ``median``  CREPE.py:179-209, then ``f0[pd < 0.1] = 0``.

``predict`` decodes each batch of ``batch_size`` frames separately (the reference's viterbi runs
per batch, CREPE.py:96-99).  librosa is absent from this image: ``viterbi`` restates librosa
>= 0.10's ``sequence.viterbi`` (log domain, uniform p_init, epsilon = tiny(dtype), first-index argmax,
value array in the probability dtype) -- "parity unpinned" for the decode; the network and
preprocessing are pinned to the reference by tests/golden/crepe.npz.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

CENTS_PER_BIN, PITCH_BINS, WINDOW_SIZE = 20, 360, 1024
CAPACITY = {
    "full": ([1, 1024, 128, 128, 128, 256], [1024, 128, 128, 128, 256, 512], 2048),
    "large": ([1, 768, 96, 96, 96, 192], [768, 96, 96, 96, 192, 384], 1536),
    "medium": ([1, 512, 64, 64, 64, 128], [512, 64, 64, 64, 128, 256], 1024),
    "small": ([1, 256, 32, 32, 32, 64], [256, 32, 32, 32, 64, 128], 512),
    "tiny": ([1, 128, 16, 16, 16, 32], [128, 16, 16, 16, 32, 64], 256),
}


def preprocess(audio: torch.Tensor, hop: int, batch_size: int):
    """audio [1, N] f32 -> list of frame batches [b, 1024] (pad=True path)."""
    total_frames = 1 + int(audio.size(1) // hop)
    audio = F.pad(audio, (WINDOW_SIZE // 2, WINDOW_SIZE // 2))
    out = []
    for i in range(0, total_frames, batch_size):
        seg = audio[:, max(0, i * hop): min(audio.size(1), (i + batch_size - 1) * hop + WINDOW_SIZE)]
        frames = seg.unfold(1, WINDOW_SIZE, hop).reshape(-1, WINDOW_SIZE).clone()
        frames -= frames.mean(dim=1, keepdim=True)
        frames /= torch.max(torch.tensor(1e-10), frames.std(dim=1, keepdim=True))
        out.append(frames)
    return out


def network(sd: dict, frames: torch.Tensor, capacity="full") -> torch.Tensor:
    """frames [b, 1024] -> sigmoid probabilities [b, 360]."""
    _, _, nfeat = CAPACITY[capacity]
    x = frames[:, None, :, None]
    for i in range(1, 7):
        pad = (0, 0, 254, 254) if i == 1 else (0, 0, 31, 32)
        x = F.conv2d(F.pad(x, pad), sd[f"conv{i}.weight"], sd[f"conv{i}.bias"], stride=(4, 1) if i == 1 else (1, 1))
        x = F.relu(x)
        x = F.batch_norm(x, sd[f"conv{i}_BN.running_mean"], sd[f"conv{i}_BN.running_var"], sd[f"conv{i}_BN.weight"],
                         sd[f"conv{i}_BN.bias"], False, 0.0, 0.0010000000474974513)
        x = F.max_pool2d(x, (2, 1), (2, 1))
    x = x.permute(0, 2, 1, 3).reshape(-1, nfeat)
    return torch.sigmoid(F.linear(x, sd["classifier.weight"], sd["classifier.bias"]))


def _transition():
    xx, yy = np.meshgrid(range(360), range(360))
    t = np.maximum(12 - abs(xx - yy), 0)
    return t / t.sum(axis=1, keepdims=True)


def viterbi_librosa(prob: np.ndarray, transition: np.ndarray) -> np.ndarray:
    """librosa.sequence.viterbi(prob [n_states, n_steps], transition) restated (see header)."""
    n_states, n_steps = prob.shape
    eps = np.finfo(prob.dtype).tiny
    log_trans = np.log(transition + np.finfo(transition.dtype).tiny)
    log_prob = np.log(prob + eps).T  # [n_steps, n_states], prob dtype
    p_init = np.full(n_states, 1.0 / n_states)
    log_p_init = np.log(p_init + np.finfo(p_init.dtype).tiny)
    value = np.zeros((n_steps, n_states), dtype=log_prob.dtype)
    ptr = np.zeros((n_steps, n_states), dtype=np.uint16)
    value[0] = log_prob[0] + log_p_init
    for t in range(1, n_steps):
        trans_out = value[t - 1] + log_trans.T  # [j][k]
        ptr[t] = np.argmax(trans_out, axis=1)
        value[t] = log_prob[t] + trans_out[np.arange(n_states), ptr[t]]
    state = np.zeros(n_steps, dtype=np.uint16)
    state[-1] = np.argmax(value[-1])
    for t in range(n_steps - 2, -1, -1):
        state[t] = ptr[t + 1, state[t + 1]]
    return state


def frequency_to_bins(frequency, quantize_fn=torch.floor):
    return quantize_fn(((1200 * torch.log2(frequency / 10)) - 1997.3794084376191) / CENTS_PER_BIN).int()


def postprocess(probabilities: torch.Tensor, fmin, fmax, dither: np.ndarray):
    """probabilities [1, 360, T] -> (pitch [1, T], periodicity [1, T]); dither [T] cents."""
    probabilities = probabilities.detach().clone()
    probabilities[:, :frequency_to_bins(torch.tensor(fmin))] = -float("inf")
    probabilities[:, frequency_to_bins(torch.tensor(fmax), torch.ceil):] = -float("inf")
    probs = torch.softmax(probabilities, dim=1)
    tr = _transition()
    bins = torch.tensor(np.array([viterbi_librosa(seq, tr).astype(np.int64) for seq in probs.numpy()]))
    cents = CENTS_PER_BIN * bins + 1997.3794084376191
    pitch = 10 * 2 ** ((cents + cents.new_tensor(dither.reshape(cents.shape))) / 1200)
    pd = probabilities.transpose(1, 2).reshape(-1, PITCH_BINS).gather(1, bins.reshape(-1, 1).to(torch.int64))
    return pitch, pd.reshape(probabilities.size(0), probabilities.size(2))


def mean(signals, win_length=9):
    signals = signals.unsqueeze(1)
    mask = ~torch.isnan(signals)
    padding = win_length // 2
    ones = torch.ones(signals.size(1), 1, win_length)
    avg = F.conv1d(torch.where(mask, signals, torch.zeros_like(signals)), ones, stride=1, padding=padding) / \
        F.conv1d(mask.float(), ones, stride=1, padding=padding).clamp(min=1)
    avg[avg == 0] = float("nan")
    return avg.squeeze(1)


def median(signals, win_length):
    signals = signals.unsqueeze(1)
    mask = ~torch.isnan(signals)
    padding = win_length // 2
    x = F.pad(torch.where(mask, signals, torch.zeros_like(signals)), (padding, padding), mode="reflect")
    mask = F.pad(mask.float(), (padding, padding), mode="constant", value=0)
    x = x.unfold(2, win_length, 1)
    mask = mask.unfold(2, win_length, 1)
    x = x.contiguous().view(x.size()[:3] + (-1,))
    mask = mask.contiguous().view(mask.size()[:3] + (-1,))
    xs, _ = torch.sort(torch.where(mask.bool(), x.float(), float("inf")).to(x), dim=-1)
    med = xs.gather(-1, ((mask.sum(dim=-1) - 1) // 2).clamp(min=0).unsqueeze(-1).long()).squeeze(-1)
    med[torch.isinf(med)] = float("nan")
    return med.squeeze(1)


def get_f0_crepe(sd, x: np.ndarray, dither: np.ndarray, capacity="full", hop=160, f0_min=50, f0_max=1100,
                 batch_size=512, trace=None):
    """VC.get_f0_crepe (convert.py:230-237) with the dither injected: x f64 [N] -> f0 f32 [1 + N//hop]."""
    audio = torch.tensor(np.copy(x))[None].float()
    pitches, pds, probs_all = [], [], []
    off = 0
    with torch.no_grad():
        for frames in preprocess(audio, hop, batch_size):
            p = network(sd, frames, capacity)
            probs_all.append(p)
            probs = p.reshape(audio.size(0), -1, PITCH_BINS).transpose(1, 2)
            n = probs.shape[-1]
            pitch, pd = postprocess(probs, f0_min, f0_max, dither[off: off + n])
            off += n
            pitches.append(pitch)
            pds.append(pd)
    f0, pd = torch.cat(pitches, 1), torch.cat(pds, 1)
    if trace is not None:
        trace.update(probs=torch.cat(probs_all).numpy(), f0_raw=f0.numpy().copy(), pd_raw=pd.numpy().copy())
    f0, pd = mean(f0, 3), median(pd, 3)
    f0[pd < 0.1] = 0
    return f0[0].cpu().numpy()
