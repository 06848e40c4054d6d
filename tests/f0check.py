"""RMVPE f0 decisions, checked against the EXACT model and the reference's own numerical noise.

RMVPE's f0 is a per-frame decision: argmax over 360 salience bins, voiced if the maximum exceeds 0.03
(RMVPE.py:217-252).  Any f32 evaluation of the network -- the reference's own at another torch thread
count, the oracle, the device -- differs from the exact (f64) evaluation by a small amount, and on the
synthetic random-init weights a few frames per clip have their top two bins (or the maximum and 0.03)
closer together than that.  Those frames' decisions are not determined at f32 precision.

The yardstick is the reference itself: ``tests/golden/ref_spread_cfg2.npz`` (``make_golden.py spread``)
ran the reference's VC.pipeline on the headline clip at 8 torch thread counts, on the input with 1-ulp
perturbations of its filtered signal (3 runs: the size of the difference between two filtfilt summation
orders), plus once with its RMVPE in float64, and holds every run's salience at the f64 run's top-2 bins per
frame.  One of the perturbed runs itself takes a different decision than f64 (frame 326, exact margin 1.7e-5)
and its waveform differs from the others by 1e-2 RMS.  From it:

  * DECISION_NOISE_MAX   the largest error of a decision quantity (top1 - top2, top1 - 0.03) any reference
                         f32 run made against f64 over the whole clip;
  * DECISION_NOISE_RMS   the largest per-run RMS of that error;
  * SAL_ERR_MAX          the largest |salience - f64 salience| of any reference run.

``check`` evaluates the device's salience and the oracle's (f32, the reference's arithmetic) against the
oracle evaluated in float64 on the same clip and asserts that the device's error is within NOISE_FACTOR of
the reference's in every statistic, and that every decision the device takes differently from the exact
model sits on a frame whose exact margin is below the smallest margin at which any reference run itself
took a different decision (FLIP_MARGIN: frame 326 of one 1-ulp-perturbed run, 1.7e-5) -- the unperturbed
reference runs take every exact decision.  Since round 4 the device's RMVPE runs in f64 (rmvpe64.hip) and
takes the exact model's decisions everywhere; ``check(..., exact=True)`` asserts that.
"""
from __future__ import annotations

import os

import numpy as np
import torch

DEV = "cuda"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_spread_cfg2.npz")
NOISE_FACTOR = 1.5


def reference_noise() -> dict:
    """The reference's own f32-vs-f64 statistics on the headline clip (the fixture above)."""
    z = np.load(GOLDEN)
    st = z["sal_top2"]  # [runs][2][F]: each run's salience at the f64 run's top-1 / top-2 bin; last = f64
    s64 = st[-1]
    d64, v64 = s64[0] - s64[1], s64[0] - 0.03
    err = [np.maximum(np.abs((r[0] - r[1]) - d64), np.abs((r[0] - 0.03) - v64)) for r in st[:-1]]
    # each f32 run's decisions different from the f64 run's (a 1-ulp input perturbation flips one frame)
    ref_flips = [np.flatnonzero((z["argmax"][i] != z["argmax"][-1]) | (z["voiced"][i] != z["voiced"][-1]))
                 for i in range(len(st) - 1)]
    same = [i for i, f in enumerate(ref_flips) if not len(f)] + [len(st) - 1]
    return dict(decision_noise_max=float(np.max(err)),
                decision_noise_rms=float(max(np.sqrt(np.mean(e ** 2)) for e in err)),
                decision_noise_frame=np.max(err, 0), sal_err_max=float(z["sal_max"][:-1, -1].max()),
                # waveform spread among the runs that take every f64 decision, and over all runs
                wav_spread=float(z["wav_rms"][np.ix_(same, same)].max()), wav_spread_all=float(z["wav_rms"].max()),
                reference_flips={str(z["names"][i]): f.tolist() for i, f in enumerate(ref_flips) if len(f)},
                # the smallest exact margin at which a reference run took a different decision
                flip_margin=float(min(z["margin64"][f].min() for f in ref_flips if len(f))),
                margin64=z["margin64"], names=[str(n) for n in z["names"]])


def oracle_salience(sd: dict, audio: np.ndarray, dtype=torch.float64) -> np.ndarray:
    """The oracle's RMVPE salience [F][360] on the reference's own input: scipy filtfilt + reflect pad
    (convert.py:403,416), in ``dtype`` (f64 = the exact model; f32 = the reference's arithmetic)."""
    from oracle import pipeline as opl
    from oracle import rmvpe as orm
    from rvc_amd import melbasis
    ap = np.pad(opl.signal.filtfilt(opl.BH, opl.AH, audio), (16000, 16000), mode="reflect")
    W = orm.load_weights(sd, dtype)
    torch.set_num_threads(16)
    with torch.no_grad():
        mel = orm.mel_spectrogram(torch.from_numpy(ap).to(dtype).unsqueeze(0), torch.from_numpy(melbasis.mel_filterbank()))
        return orm.mel2hidden(W, mel).squeeze(0).numpy().astype(np.float64)


def decision_noise(s: np.ndarray, s64: np.ndarray) -> np.ndarray:
    """Per frame: the error of the two quantities the decision compares, at the exact model's top-2 bins."""
    fi = np.arange(s64.shape[0])
    top = np.argsort(s64, 1)[:, -2:]
    a, b = top[:, 1], top[:, 0]
    return np.maximum(np.abs((s[fi, a] - s[fi, b]) - (s64[fi, a] - s64[fi, b])), np.abs(s[fi, a] - s64[fi, a]))


def margins(s64: np.ndarray) -> np.ndarray:
    srt = np.sort(s64, 1)
    return np.minimum(srt[:, -1] - srt[:, -2], np.abs(srt[:, -1] - 0.03))


def flips(s: np.ndarray, s64: np.ndarray) -> np.ndarray:
    return np.flatnonzero((s.argmax(1) != s64.argmax(1)) | ((s.max(1) > 0.03) != (s64.max(1) > 0.03)))


def device_salience(vc, audio: np.ndarray):
    """The device's salience [F][360] and raw f0 track (f64 [F]) for one clip, through VC's own filtfilt."""
    xp, _ = vc.filt(torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32)).to(DEV), vc.t_pad)
    mel = vc.rmvpe.mel_spectrogram(xp)
    F = mel.shape[-1]
    sal, _ = vc.rmvpe.salience(mel)
    _, _, f0 = vc.rmvpe.f0_device(xp, 0.03, 0.0, want_f0=True)
    vc.check_errors()
    return sal[:, :F].t().cpu().numpy().astype(np.float64), f0.cpu().numpy()


def check(vc, sd: dict, audio: np.ndarray, factor: float = NOISE_FACTOR, max_flip_frac: float = 1e-3,
          device=None, exact=None):
    """Device RMVPE on one clip vs the exact model, within ``factor`` of the reference's own f32 noise.
    ``device`` = (salience [F][360], raw f0 [F]) the caller computed (e.g. by the batched path), else the
    per-clip device path's.  ``exact`` (default: when the model runs in f64) also requires every decision to
    equal the exact model's.  Returns (device raw f0, exact-model raw f0, report)."""
    if exact is None:
        exact = bool(getattr(getattr(vc, "rmvpe", None), "f64", False))
    from oracle import rmvpe as orm
    ref = reference_noise()
    sdv, f0_dev = device if device is not None else device_salience(vc, audio)
    s64 = oracle_salience(sd, audio, torch.float64)
    s32 = oracle_salience(sd, audio, torch.float32)
    F = s64.shape[0]
    m = margins(s64)
    nd, no = decision_noise(sdv, s64), decision_noise(s32, s64)
    fl = flips(sdv, s64)
    rep = dict(frames=int(F), sal_err_max=float(np.abs(sdv - s64).max()),
               sal_err_max_oracle_f32=float(np.abs(s32 - s64).max()), sal_err_max_reference=ref["sal_err_max"],
               decision_noise_max=float(nd.max()), decision_noise_rms=float(np.sqrt(np.mean(nd ** 2))),
               decision_noise_max_oracle_f32=float(no.max()),
               decision_noise_rms_oracle_f32=float(np.sqrt(np.mean(no ** 2))),
               decision_noise_max_reference=ref["decision_noise_max"],
               decision_noise_rms_reference=ref["decision_noise_rms"],
               flips_vs_exact=fl.tolist(), flip_margins=m[fl].tolist(),
               flips_oracle_f32_vs_exact=flips(s32, s64).tolist(),
               frames_below_reference_noise=np.flatnonzero(m < ref["decision_noise_max"]).size)
    assert rep["sal_err_max"] <= factor * max(ref["sal_err_max"], rep["sal_err_max_oracle_f32"]), rep
    assert rep["decision_noise_max"] <= factor * max(ref["decision_noise_max"], rep["decision_noise_max_oracle_f32"]), rep
    assert rep["decision_noise_rms"] <= factor * max(ref["decision_noise_rms"], rep["decision_noise_rms_oracle_f32"]), rep
    # a decision unlike the exact model's only where a reference run itself took one (below FLIP_MARGIN)
    rep["flip_margin_reference"] = ref["flip_margin"]
    assert all(m[fl] < ref["flip_margin"]), rep
    assert len(fl) <= max(2, int(F * max_flip_frac)), rep
    if exact:
        assert not len(fl), rep
    f0_64 = orm.decode(s64, thred=0.03)
    return f0_dev, f0_64, rep


def _rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


def assert_pipeline(vc, out, sd: dict, audio: np.ndarray, oracle_fn, tol: float = 1e-4):
    """A whole VC.pipeline output against the oracle: the f0 decisions by ``check``, then the waveform against
    ``oracle_fn(f0_track)`` (the oracle pipeline with that raw f0) on the device's own decisions and -- when
    every decision equals the exact model's -- on the exact model's, both within ``tol`` RMS.
    Returns (rms on the device f0, rms on the exact f0 or None, f0 report)."""
    f0_dev, f0_64, rep = check(vc, sd, audio)
    ref = oracle_fn(f0_dev)
    assert out.shape == ref.shape, (out.shape, ref.shape)
    err = _rms(out, ref)
    assert err < tol, (err, rep)
    err_exact = None
    if not rep["flips_vs_exact"]:
        err_exact = _rms(out, oracle_fn(f0_64))
        assert err_exact < tol, (err_exact, rep)
    return err, err_exact, rep
