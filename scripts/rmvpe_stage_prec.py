"""Which RMVPE stages need f64 for the exact model's f0 decisions: the oracle's RMVPE evaluated in
float64 with ONE stage at a time run in float32 (torch-CPU f32: the reference's arithmetic; the device's
split-accumulator f32 convs measured ~1.7x closer to f64 on the U-Net), on the 30 s headline clip.
For every frame the decision quantities are the exact model's top-1 minus top-2 salience (at the exact top-2 bins)
and top-1 minus the 0.03 voicing threshold; a stage's "decision noise" is the largest change it makes to either,
over all frames.  A stage whose noise stays below the smallest exact margin of the clip (3.2e-6 at frame 721 here)
with a wide factor could leave f64.

    python scripts/rmvpe_stage_prec.py [seconds] [--stages mel,enc0,...] [--out profiles/r5_rmvpe_stage_prec.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
sys.path.insert(0, REPO)

from oracle import rmvpe as orm  # noqa: E402

STAGES = ["mel", "enc_bn"] + [f"enc{l}" for l in range(5)] + [f"int{l}" for l in range(4)] + \
         [f"dec{l}" for l in range(5)] + ["cnn", "w_ih", "gru", "fc"]


def run(W64, W32, mel64, mel32, low):
    """Salience [T][360] (f64) with the stages in ``low`` evaluated in f32."""
    def W(stage):
        return W32 if stage in low else W64

    def cast(x, stage):
        return x.float() if stage in low else x.double()

    x = (mel32 if "mel" in low else mel64).double()
    n = x.shape[-1]
    x = F.pad(x, (0, 32 * ((n - 1) // 32 + 1) - n), mode="reflect").transpose(-1, -2).unsqueeze(1)
    x = orm._bn(W("enc_bn"), "unet.encoder.bn", cast(x, "enc_bn")).double()
    skips = []
    for l in range(5):
        s = f"enc{l}"
        x = cast(x, s)
        for b in range(4):
            x = orm._cbr(W(s), f"unet.encoder.layers.{l}.conv.{b}", x)
        skips.append(x.double())
        x = F.avg_pool2d(x, 2).double()
    for l in range(4):
        s = f"int{l}"
        x = cast(x, s)
        for b in range(4):
            x = orm._cbr(W(s), f"unet.intermediate.layers.{l}.conv.{b}", x)
        x = x.double()
    for l in range(5):
        s, p = f"dec{l}", f"unet.decoder.layers.{l}"
        x = cast(x, s)
        Ws = W(s)
        x = F.conv_transpose2d(x, Ws[p + ".conv1.0.weight"], None, (2, 2), (1, 1), (1, 1))
        x = F.relu(orm._bn(Ws, p + ".conv1.1", x))
        x = torch.cat((x, cast(skips[-1 - l], s)), dim=1)
        for b in range(4):
            x = orm._cbr(Ws, f"{p}.conv2.{b}", x)
        x = x.double()
    x = cast(x, "cnn")
    x = F.conv2d(x, W("cnn")["cnn.weight"], W("cnn")["cnn.bias"], 1, 1).double()
    x = x.transpose(1, 2).flatten(-2)[0]  # [T][384]
    pre = "fc.0.gru."
    outs = []
    for sfx, rev in (("", False), ("_reverse", True)):
        Wi = W("w_ih")
        gi = F.linear(cast(x, "w_ih"), Wi[pre + "weight_ih_l0" + sfx], Wi[pre + "bias_ih_l0" + sfx]).double()
        Wg = W("gru")
        w_hh, b_hh = Wg[pre + "weight_hh_l0" + sfx], Wg[pre + "bias_hh_l0" + sfx]
        gi = cast(gi, "gru")
        H = w_hh.shape[1]
        h = torch.zeros(H, dtype=gi.dtype)
        out = torch.empty(gi.shape[0], H, dtype=gi.dtype)
        for t in (range(gi.shape[0] - 1, -1, -1) if rev else range(gi.shape[0])):
            gh = F.linear(h, w_hh, b_hh)
            r = torch.sigmoid(gi[t, :H] + gh[:H])
            z = torch.sigmoid(gi[t, H:2 * H] + gh[H:2 * H])
            nn_ = torch.tanh(gi[t, 2 * H:] + r * gh[2 * H:])
            h = (h - nn_) * z + nn_
            out[t] = h
        outs.append(out.double())
    x = torch.cat(outs, -1)
    x = cast(x, "fc")
    return torch.sigmoid(F.linear(x, W("fc")["fc.1.weight"], W("fc")["fc.1.bias"])).double()[:n].numpy()


def decision_noise(sal, ex):
    """Largest change of the exact model's decision quantities (top1 - top2 at the exact bins; top1 - 0.03)."""
    order = np.argsort(-ex, axis=1)
    a, b = order[:, 0], order[:, 1]
    r = np.arange(len(ex))
    d = sal - ex
    dm = d[r, a] - d[r, b]
    dt = d[r, a]
    margins = np.minimum(ex[r, a] - ex[r, b], np.abs(ex[r, a] - 0.03))
    return {"max": float(max(np.abs(dm).max(), np.abs(dt).max())),
            "rms": float(np.sqrt(np.mean(np.concatenate([dm, dt]) ** 2))),
            "sal_err_max": float(np.abs(d).max()),
            "flips": int(np.sum((np.abs(dm) > (ex[r, a] - ex[r, b])) | (np.abs(dt) > np.abs(ex[r, a] - 0.03)))),
            "min_margin": float(margins.min())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("seconds", nargs="?", type=float, default=30.0)
    ap.add_argument("--stages", default=",".join(["all32"] + STAGES))
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--out", default="")
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    from oracle import pipeline as opl
    from rvc_amd import melbasis, synthetic
    sd = synthetic.rmvpe_state_dict(args.seed + 2)  # the headline bench's RMVPE weights (bench.build_models)
    W32, W64 = orm.load_weights(sd), orm.load_weights(sd, torch.float64)
    audio = synthetic.synthetic_audio(args.seconds, seed=1000)
    ap_ = np.pad(opl.signal.filtfilt(opl.BH, opl.AH, audio), (16000, 16000), mode="reflect")
    mb = torch.from_numpy(melbasis.mel_filterbank())
    with torch.no_grad():
        # the reference hands RMVPE f32 audio (RMVPE.py:224): both arms start from the f32-rounded signal
        a32 = torch.from_numpy(ap_.astype(np.float32))
        mel64 = orm.mel_spectrogram(a32.double().unsqueeze(0), mb)
        mel32 = orm.mel_spectrogram(a32.unsqueeze(0), mb)
        t0 = time.time()
        ex = run(W64, W32, mel64, mel32, set())
        print(f"exact (f64) pass {time.time() - t0:.1f} s, frames {len(ex)}", flush=True)
        res = {}
        for st in args.stages.split(","):
            low = set(STAGES) if st == "all32" else {st}
            t0 = time.time()
            sal = run(W64, W32, mel64, mel32, low)
            res[st] = decision_noise(sal, ex)
            print(f"{st:8s} decision noise max {res[st]['max']:.3e} rms {res[st]['rms']:.3e}  salience err max "
                  f"{res[st]['sal_err_max']:.3e}  flips {res[st]['flips']}  ({time.time() - t0:.0f} s)", flush=True)
    out = {"seconds": args.seconds, "min_exact_margin": decision_noise(ex, ex)["min_margin"],
           "arithmetic": "torch-CPU f32 for the named stage, f64 elsewhere (oracle/rmvpe.py)", "stages": res}
    print(json.dumps({"min_exact_margin": out["min_exact_margin"]}))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
