"""Where does the device f0 leave the oracle's?  RMVPE salience on the device vs the oracle (CPU) for one
clip: voicing flips, argmax moves, and the margins (max - threshold, top1 - top2) at those frames.

    python scripts/f0_diag.py [seconds] [seed]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
sys.path.insert(0, REPO)


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 30.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 201
    from oracle import rmvpe as orm
    from oracle import pipeline as opl
    from rvc_amd import melbasis, synthetic
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    dev = "cuda"
    sd = synthetic.rmvpe_state_dict(seed + 2)
    m = RMVPEAMD(sd, dev)
    vc = VC(48000, Config(dev), rmvpe=m)
    audio = synthetic.synthetic_audio(secs, seed=1000)
    xp, _ = vc.filt(torch.from_numpy(audio).to(dev), vc.t_pad)
    mel = m.mel_spectrogram(xp)
    sal, Tp = m.salience(mel)
    F = mel.shape[-1]
    sd_dev = sal[:, :F].t().cpu().numpy().astype(np.float64)  # [F][360]
    # oracle on the oracle's own filtered/padded signal
    a = opl.signal.filtfilt(opl.BH, opl.AH, audio)
    ap = np.pad(a, (16000, 16000), mode="reflect")
    torch.set_num_threads(16)
    W = orm.load_weights(sd)
    mb = torch.from_numpy(melbasis.mel_filterbank())
    with torch.no_grad():
        melo = orm.mel_spectrogram(torch.from_numpy(ap).float().unsqueeze(0), mb)
        so = orm.mel2hidden(W, melo).squeeze(0).numpy().astype(np.float64)  # [F][360]
    print(f"frames {F}; mel rms diff {float((mel.cpu() - melo[0]).pow(2).mean().sqrt()):.3e}; "
          f"salience max abs diff {np.abs(sd_dev - so).max():.3e}")
    fd, fo = orm.decode(sd_dev.astype(np.float32), 0.03), orm.decode(so.astype(np.float32), 0.03)
    vd, vo = fd > 0, fo > 0
    print(f"voiced frames dev {vd.sum()} oracle {vo.sum()}; voicing flips {int((vd != vo).sum())}")
    am_d, am_o = sd_dev.argmax(1), so.argmax(1)
    print(f"argmax moves {int((am_d != am_o).sum())}; f0 |diff| > 1 cent on {int((np.abs(1200 * np.log2((fd + 1e-9) / (fo + 1e-9))) > 1).sum())} frames")
    srt = np.sort(so, axis=1)
    top_gap = srt[:, -1] - srt[:, -2]
    print(f"oracle salience: max median {np.median(srt[:, -1]):.4f}, top1-top2 gap median {np.median(top_gap):.3e}, "
          f"frames with gap < 1e-5: {int((top_gap < 1e-5).sum())}, |max - 0.03| < 1e-5: "
          f"{int((np.abs(srt[:, -1] - 0.03) < 1e-5).sum())}")
    for t in np.flatnonzero((am_d != am_o) | (vd != vo))[:12]:
        print(f"  t={t}: argmax dev {am_d[t]} oracle {am_o[t]} gap {top_gap[t]:.3e} max {srt[t, -1]:.5f} "
              f"f0 dev {fd[t]:.2f} oracle {fo[t]:.2f}")


if __name__ == "__main__":
    main()
