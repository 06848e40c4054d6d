"""pm f0 restatement (oracle/pm.py: Praat's To Pitch (ac) as VC.get_f0_pm calls it, convert.py:206-213) on
known pitch tracks.  Parity against Praat itself is unpinned: parselmouth is not installed."""
import math

import numpy as np

from oracle import pm


def vibrato(seconds=1.5, f=150.0, depth=0.1, rate=1.5, lead=0.5, tail=0.25, sr=16000, noise=1e-4, seed=0):
    t = np.arange(int(seconds * sr)) / sr
    inst = f * (1 + depth * np.sin(2 * np.pi * rate * t))
    ph = 2 * np.pi * np.cumsum(inst) / sr
    x = 0.5 * np.sin(ph) + 0.2 * np.sin(2 * ph) + 0.1 * np.sin(3 * ph)
    x = np.concatenate([np.zeros(int(lead * sr)), x, np.zeros(int(tail * sr))])
    x += noise * np.random.default_rng(seed).standard_normal(len(x))
    truth = lambda tt: f * (1 + depth * np.sin(2 * np.pi * rate * (tt - lead)))  # noqa: E731
    return x, truth


def test_geometry_matches_praat_frame_grid():
    for n in (16000, 80000, 80160, 123457):
        g = pm.geometry(n)
        dur = n / 16000
        assert g["nframes"] == math.floor((dur - 0.06) / 0.01) + 1
        # frames are centred: the first window starts within one sample of the signal start
        assert abs((g["t1"] - 0.03) - (dur - (g["t1"] + (g["nframes"] - 1) * 0.01 + 0.03))) < 1e-9
        assert (g["nsamp_window"], g["brent_ixmax"], g["maximum_lag"]) == (958, 479, 321)


def test_tracks_vibrato_and_silence():
    x, truth = vibrato()
    f0 = pm.to_pitch_ac(x)
    g = pm.geometry(len(x))
    tt = g["t1"] + np.arange(g["nframes"]) * g["dt"]
    inside = (tt > 0.55) & (tt < 1.95)
    assert np.all(f0[inside] > 0)
    assert np.max(np.abs(f0[inside] / truth(tt[inside]) - 1)) < 1e-3
    assert np.all(f0[(tt < 0.45) | (tt > 2.05)] == 0)


def test_octave_and_range():
    # 90 Hz with a strong 2nd harmonic stays at 90 (octave cost), 700 Hz is tracked (ceiling 1100)
    for f in (90.0, 700.0):
        x, truth = vibrato(seconds=1.0, f=f, depth=0.0, lead=0.1, tail=0.1)
        f0 = pm.to_pitch_ac(x)
        mid = f0[len(f0) // 3: 2 * len(f0) // 3]
        assert np.all(np.abs(mid / f - 1) < 1e-3), (f, mid[:5])


def test_get_f0_pm_pads_to_p_len():
    x, _ = vibrato(seconds=0.5, lead=0.1, tail=0.1)
    p_len = len(x) // 160
    f0 = pm.get_f0_pm(x, p_len)
    nf = pm.geometry(len(x))["nframes"]
    assert len(f0) == p_len and nf < p_len
    pad = (p_len - nf + 1) // 2
    assert np.array_equal(f0[pad: pad + nf], pm.to_pitch_ac(x))
    assert np.all(f0[:pad] == 0) and np.all(f0[pad + nf:] == 0)
