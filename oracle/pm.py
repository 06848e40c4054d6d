"""TEST INFRASTRUCTURE ONLY (the checker, never the product path): numpy restatement of the pm f0 method,
VC.get_f0_pm (main/inference/convert.py:206-213):

    parselmouth.Sound(x, 16000).to_pitch_ac(time_step=0.01, voicing_threshold=0.6, pitch_floor=50,
                                            pitch_ceiling=1100).selected_array["frequency"]
    zero-padded to p_len, (p_len - n + 1) // 2 frames in front

i.e. Praat's "To Pitch (ac)" (praat-parselmouth, requirements.txt:28; Praat's Sound_to_Pitch.cpp
Sound_to_Pitch_any with method AC_HANNING, Pitch_pathFinder, NUM_interpolate_sinc, NUMimproveMaximum /
NUMminimize_brent) with its remaining defaults: 15 candidates, silence threshold 0.03, octave cost 0.01,
octave-jump cost 0.35, voiced/unvoiced cost 0.14, 3 periods per window, not "very accurate".  The
algorithm is Boersma (1993), "Accurate short-term analysis of the fundamental frequency and the
harmonics-to-noise ratio of a sampled sound", as Praat implements it; it is restated here from that
published algorithm because parselmouth is not installed: PARITY UNPINNED (no golden from Praat itself).
Praat's FFT autocorrelation is computed directly (the zero padding to 2048 >= 958 + 479 samples makes it
the linear autocorrelation for every lag used), equal up to f64 rounding.
"""
from __future__ import annotations

import math

import numpy as np

PM = dict(time_step=160 / 16000 * 1000 / 1000, pitch_floor=50.0, pitch_ceiling=1100.0, max_candidates=15,
          silence_threshold=0.03, voicing_threshold=0.6, octave_cost=0.01, octave_jump_cost=0.35,
          voiced_unvoiced_cost=0.14, periods_per_window=3.0)


def geometry(nx, sr=16000, floor=50.0, ceiling=1100.0, dt=PM["time_step"], periods=3.0):
    """Sound_to_Pitch_any's sizes and Sampled_shortTermAnalysis's frame grid (Praat, 1-based sample
    numbers converted to 0-based here)."""
    dx = 1.0 / sr
    x1 = 0.5 * dx  # time of the first sample of parselmouth.Sound(array, sr)
    nsamp_period = int(math.floor(1.0 / dx / floor))
    halfnsamp_period = nsamp_period // 2 + 1
    ceiling = min(ceiling, 0.5 / dx)
    dt_window = periods / floor
    nsamp_window = int(math.floor(dt_window / dx))
    halfnsamp_window = nsamp_window // 2 - 1
    nsamp_window = halfnsamp_window * 2
    maximum_lag = min(int(math.floor(nsamp_window / periods)) + 2, nsamp_window)
    duration = dx * nx
    if dt_window > duration:
        raise ValueError("pm: the sound is shorter than one analysis window (60 ms)")
    nframes = int(math.floor((duration - dt_window) / dt)) + 1
    mid = x1 - 0.5 * dx + 0.5 * duration
    t1 = mid - 0.5 * nframes * dt + 0.5 * dt
    brent_ixmax = int(math.floor(nsamp_window * 0.5))
    return dict(dx=dx, x1=x1, nsamp_period=nsamp_period, halfnsamp_period=halfnsamp_period, ceiling=ceiling,
                nsamp_window=nsamp_window, halfnsamp_window=halfnsamp_window, maximum_lag=maximum_lag,
                nframes=nframes, t1=t1, dt=dt, brent_ixmax=brent_ixmax)


def hanning(n):
    i = np.arange(1, n + 1, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(i * 2 * np.pi / (n + 1))


def autocorr(v, nlag):
    """linear autocorrelation v (x) v at lags 0..nlag (numpy dot per lag, f64)."""
    n = len(v)
    return np.array([float(np.dot(v[:n - i], v[i:])) for i in range(nlag + 1)])


def sinc_interp(y, x, max_depth):
    """NUM_interpolate_sinc: y is 1-based in Praat (y[1..n]); here y[0] is Praat's y[1], x Praat's 1-based x."""
    n = len(y)
    ix = int(math.floor(x))
    if x > n:
        return y[n - 1]
    if x < 1:
        return y[0]
    if x == ix:
        return y[ix - 1]
    midleft, midright = ix, ix + 1
    max_depth = min(max_depth, midright - 1, n - midleft)
    left, right = midright - max_depth, midleft + max_depth
    result = 0.0
    a = math.pi * (x - midleft)
    halfsina = 0.5 * math.sin(a)
    aa = a / (x - left + 1.0)
    daa = math.pi / (x - left + 1.0)
    for i in range(midleft, left - 1, -1):
        result += y[i - 1] * (halfsina / a * (1.0 + math.cos(aa)))
        a += math.pi
        aa += daa
        halfsina = -halfsina
    a = math.pi * (midright - x)
    halfsina = 0.5 * math.sin(a)
    aa = a / (right - x + 1.0)
    daa = math.pi / (right - x + 1.0)
    for i in range(midright, right + 1):
        result += y[i - 1] * (halfsina / a * (1.0 + math.cos(aa)))
        a += math.pi
        aa += daa
        halfsina = -halfsina
    return result


def brent_min(f, a, b, tol=1e-10, itermax=60):
    """NUMminimize_brent (Brent's fmin): -> (xmin, fmin)."""
    golden = 0.3819660112501051
    sqrt_eps = math.sqrt(np.finfo(np.float64).eps)
    v = a + golden * (b - a)
    fv = f(v)
    x = w = v
    fx = fw = fv
    for _ in range(itermax):
        middle = (a + b) / 2.0
        tol_act = sqrt_eps * abs(x) + tol / 3.0
        if abs(x - middle) + (b - a) / 2.0 <= 2.0 * tol_act:
            return x, fx
        new_step = golden * (b - x if x < middle else a - x)
        if abs(x - w) >= tol_act:
            t = (x - w) * (fx - fv)
            q = (x - v) * (fx - fw)
            p = (x - v) * q - (x - w) * t
            q = 2.0 * (q - t)
            if q > 0.0:
                p = -p
            else:
                q = -q
            if abs(p) < abs(new_step * q) and p > q * (a - x + 2.0 * tol_act) and p < q * (b - x - 2.0 * tol_act):
                new_step = p / q
        if abs(new_step) < tol_act:
            new_step = tol_act if new_step > 0.0 else -tol_act
        t = x + new_step
        ft = f(t)
        if ft <= fx:
            if t < x:
                b = x
            else:
                a = x
            v, w, x = w, x, t
            fv, fw, fx = fw, fx, ft
        else:
            if t < x:
                a = t
            else:
                b = t
            if ft <= fw or w == x:
                v, w = w, t
                fv, fw = fw, ft
            elif ft <= fv or v == x or v == w:
                v, fv = t, ft
    return x, fx


def frame_candidates(x, g, iframe, window, window_r, global_peak, p=PM):
    """Sound_into_PitchFrame (AC): (intensity, [(frequency, strength)] with the voiceless candidate first)."""
    dx, hw, hp, nsp = g["dx"], g["halfnsamp_window"], g["halfnsamp_period"], g["nsamp_period"]
    nw, bix = g["nsamp_window"], g["brent_ixmax"]
    t = g["t1"] + iframe * g["dt"]
    left = int(math.floor((t - g["x1"]) / dx)) + 1  # Sampled_xToLowIndex, 1-based
    right = left + 1
    mean = float(np.sum(x[right - nsp - 1: left + nsp])) / (2 * nsp)  # samples right-nsp .. left+nsp (1-based)
    seg = x[right - hw - 1: right - hw - 1 + nw]
    frame = (seg - mean) * window
    s0, s1 = max(1, hw + 1 - hp), min(nw, hw + hp)
    local_peak = float(np.max(np.abs(frame[s0 - 1: s1])))
    intensity = 1.0 if local_peak > global_peak else local_peak / global_peak
    cands = [(0.0, 0.0)]
    if local_peak == 0.0:
        return intensity, cands
    ac = autocorr(frame, bix)
    r = np.empty(2 * bix + 1)  # Praat's r[-bix..bix]; r[k] at index k + bix
    r[bix] = 1.0
    for i in range(1, bix + 1):
        r[bix + i] = r[bix - i] = ac[i] / (ac[0] * window_r[i])
    rr = lambda i: r[bix + i]  # noqa: E731
    offset = -bix - 1  # Praat's y index = lag - offset
    imax = [0]
    vt, oc, floor = p["voicing_threshold"], p["octave_cost"], p["pitch_floor"]
    for i in range(2, min(g["maximum_lag"], bix)):
        if rr(i) > 0.5 * vt and rr(i) > rr(i - 1) and rr(i) >= rr(i + 1):
            dr = 0.5 * (rr(i + 1) - rr(i - 1))
            d2r = 2.0 * rr(i) - rr(i - 1) - rr(i + 1)
            freq = 1.0 / dx / (i + dr / d2r)
            strength = sinc_interp(r, 1.0 / dx / freq - offset, 30)
            if strength > 1.0:
                strength = 1.0 / strength
            place = None
            if len(cands) < p["max_candidates"]:
                cands.append(None)
                imax.append(0)
                place = len(cands) - 1
            else:
                weakest = 2.0
                for iw in range(1, p["max_candidates"]):
                    ls = cands[iw][1] - oc * math.log2(floor / cands[iw][0])
                    if ls < weakest:
                        weakest, place = ls, iw
                if strength - oc * math.log2(floor / freq) <= weakest:
                    place = None
            if place is not None:
                cands[place] = (freq, strength)
                imax[place] = i
    for k in range(1, len(cands)):
        f, s = cands[k]
        if f > 0.0:
            depth = 700 if f > 0.3 / dx else 70
            xmid, fmin = brent_min(lambda xx: -sinc_interp(r, xx, depth), imax[k] - offset - 1,
                                   imax[k] - offset + 1)
            ymid = -fmin
            xmid += offset
            if ymid > 1.0:
                ymid = 1.0 / ymid
            cands[k] = (1.0 / dx / xmid, ymid)
    return intensity, cands


def path_finder(frames, g, p=PM):
    """Pitch_pathFinder: Viterbi over each frame's candidates -> selected frequency per frame (0 = unvoiced)."""
    ceiling, vt, oc = g["ceiling"], p["voicing_threshold"], p["octave_cost"]
    corr = 0.01 / g["dt"]
    ojc, vuc = p["octave_jump_cost"] * corr, p["voiced_unvoiced_cost"] * corr
    st = p["silence_threshold"]
    voiced = lambda f: f > 0.0 and f < ceiling  # noqa: E731
    deltas, psis = [], []
    for intensity, cands in frames:
        us = 0.0 if st <= 0 else 2.0 - intensity / (st / (1.0 + vt))
        us = vt + (us if us > 0 else 0.0)
        deltas.append([us if not voiced(f) else s - oc * math.log2(ceiling / f) for f, s in cands])
        psis.append([0] * len(cands))
    for i in range(1, len(frames)):
        prev, cur = frames[i - 1][1], frames[i][1]
        pd, cd = deltas[i - 1], deltas[i]
        new = []
        for j2, (f2, _) in enumerate(cur):
            best, place = -1e30, 0
            for j1, (f1, _) in enumerate(prev):
                if not voiced(f2):
                    tc = 0.0 if not voiced(f1) else vuc
                else:
                    tc = vuc if not voiced(f1) else ojc * abs(math.log2(f1 / f2))
                v = pd[j1] - tc + cd[j2]
                if v > best:
                    best, place = v, j1
            new.append(best)
            psis[i][j2] = place
        deltas[i] = new
    last = deltas[-1]
    place = max(range(len(last)), key=lambda j: (last[j], -j))  # first maximum
    out = np.zeros(len(frames))
    for i in range(len(frames) - 1, -1, -1):
        f = frames[i][1][place][0]
        out[i] = f if voiced(f) else 0.0
        place = psis[i][place]
    return out


def to_pitch_ac(x, sr=16000):
    """The selected frequencies of Praat's To Pitch (ac) with get_f0_pm's settings (f64 [nframes])."""
    x = np.asarray(x, dtype=np.float64)
    g = geometry(len(x), sr)
    window = hanning(g["nsamp_window"])
    wr = autocorr(window, g["brent_ixmax"])
    window_r = wr / wr[0]
    global_peak = float(np.max(np.abs(x - np.sum(x) / len(x))))
    if global_peak == 0.0:
        return np.zeros(g["nframes"])
    frames = [frame_candidates(x, g, i, window, window_r, global_peak) for i in range(g["nframes"])]
    return path_finder(frames, g)


def get_f0_pm(x, p_len, sr=16000):
    """VC.get_f0_pm (convert.py:206-213)."""
    f0 = to_pitch_ac(x, sr)
    pad = (p_len - len(f0) + 1) // 2
    if pad > 0 or p_len - len(f0) - pad > 0:
        f0 = np.pad(f0, [[pad, p_len - len(f0) - pad]], mode="constant")
    return f0
