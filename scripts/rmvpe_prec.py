"""RMVPE salience error, stage by stage: the device (f32-accurate split-bf16 convs, f32 BiGRU) and the torch-CPU
oracle in f32 (the reference's arithmetic), each measured against the oracle evaluated in float64 -- at every
stage fed the SAME f64 input, so each stage's own error is isolated:

  mel      filtered padded audio (f64, scipy)             -> log-mel [128][F]
  unet     the f64 log-mel                                -> cnn head rows / GRU input [Tp][384]
  head     the f64 GRU input                              -> salience [Tp][360] (W_ih, BiGRU, fc, sigmoid)
  chain    audio                                          -> salience (every stage's error compounded)

    python scripts/rmvpe_prec.py [seconds] [seed]
"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
sys.path.insert(0, REPO)


def _err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return f"max {np.abs(a - b).max():.3e} rms {np.sqrt(np.mean((a - b) ** 2)):.3e} (ref rms {np.sqrt(np.mean(b ** 2)):.3e})"


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 30.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 201
    from oracle import pipeline as opl
    from oracle import rmvpe as orm
    from rvc_amd import melbasis, ops, synthetic
    from rvc_amd.rmvpe import RMVPEAMD
    torch.set_num_threads(16)
    dev = "cuda"
    sd = synthetic.rmvpe_state_dict(seed + 2)
    m = RMVPEAMD(sd, dev)
    audio = synthetic.synthetic_audio(secs, seed=1000)
    ap = np.pad(opl.signal.filtfilt(opl.BH, opl.AH, audio), (16000, 16000), mode="reflect")
    mb = torch.from_numpy(melbasis.mel_filterbank())
    W32, W64 = orm.load_weights(sd), orm.load_weights(sd, torch.float64)
    t0 = time.time()
    with torch.no_grad():
        mel64 = orm.mel_spectrogram(torch.from_numpy(ap).unsqueeze(0), mb)  # [1][128][F] f64
        mel32 = orm.mel_spectrogram(torch.from_numpy(ap).float().unsqueeze(0), mb)
    F = mel64.shape[-1]
    Tp = 32 * ((F - 1) // 32 + 1)
    with ops.precision(m.precision):
        meld = m.mel_spectrogram(torch.from_numpy(ap).float().to(dev)).cpu()
    print(f"[mel] F={F}  device vs f64: {_err(meld, mel64[0])}")
    print(f"[mel]          oracle f32 vs f64: {_err(mel32[0], mel64[0])}")

    def seq_of(W, mel):
        mel = torch.nn.functional.pad(mel, (0, Tp - F), mode="reflect")
        x = orm.unet(W, mel.transpose(-1, -2).unsqueeze(1))
        x = torch.nn.functional.conv2d(x, W["cnn.weight"], W["cnn.bias"], 1, 1)
        return x.transpose(1, 2).flatten(-2)  # [1][Tp][384]

    def head_of(W, seq):
        x = orm.bigru_torch(W, seq)
        return torch.sigmoid(torch.nn.functional.linear(x, W["fc.1.weight"], W["fc.1.bias"]))

    with torch.no_grad():
        seq64 = seq_of(W64, mel64)
        seq32 = seq_of(W32, mel64.float())
    with ops.precision(m.precision):
        x, _ = m.mel_image(mel64[0].float().to(dev))
        seqd = m.unet_seq(x, Tp).cpu().t()  # [Tp][384]
    print(f"[unet] device vs f64: {_err(seqd, seq64[0])}")
    print(f"[unet]          oracle f32 vs f64: {_err(seq32[0], seq64[0])}")
    with torch.no_grad():
        sal64 = head_of(W64, seq64)[0]
        sal32h = head_of(W32, seq64.float())[0]
    with ops.precision(m.precision):
        sald = m.head(seq64[0].t().contiguous().float().to(dev)).cpu().t()
    m.check_error()
    print(f"[head] device vs f64: {_err(sald, sal64)}")
    print(f"[head]          oracle f32 vs f64: {_err(sal32h, sal64)}")
    # the GRU alone: W_ih GEMM on the device from the same input, recurrence compared through the head
    with torch.no_grad():
        sal32 = orm.mel2hidden(W32, mel32)[0]
    with ops.precision(m.precision):
        salc, _ = m.salience(m.mel_spectrogram(torch.from_numpy(ap).float().to(dev)))
    salc = salc.cpu().t()[:F]
    print(f"[chain] device vs f64: {_err(salc, sal64[:F])}")
    print(f"[chain]          oracle f32 vs f64: {_err(sal32, sal64[:F])}")
    print(f"[chain]          device vs oracle f32: {_err(salc, sal32)}")
    s64 = sal64[:F].numpy()
    srt = np.sort(s64, 1)
    margin = np.minimum(srt[:, -1] - srt[:, -2], np.abs(srt[:, -1] - 0.03))
    top = np.argsort(s64, 1)[:, -2:]
    fi = np.arange(F)
    d64 = s64[fi, top[:, 1]] - s64[fi, top[:, 0]]
    for name, s in (("device", salc.numpy()), ("oracle f32", sal32.numpy())):
        fl = np.flatnonzero((s.argmax(1) != s64.argmax(1)) | ((s.max(1) > 0.03) != (s64.max(1) > 0.03)))
        # decision noise: error of (top1 - top2) and of top1 (vs the voicing threshold) at the f64 top-2 bins
        e = np.maximum(np.abs((s[fi, top[:, 1]] - s[fi, top[:, 0]]) - d64), np.abs(s[fi, top[:, 1]] - s64[fi, top[:, 1]]))
        print(f"[decisions] {name} vs f64: flips at {fl.tolist()} margins(f64) {margin[fl].tolist()}; decision noise "
              f"max {e.max():.3e} rms {np.sqrt(np.mean(e ** 2)):.3e}; at 326/721/918/977: {e[[326, 721, 918, 977]]}")
    print(f"oracle time {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
