"""Spectral-gate denoise on the device (csrc/denoise.hip) against the reference's own output
(tests/golden/denoise.npz: noisereduce.reduce_noise run in the survey container) and the f64 oracle
at the convert_audio size (30 s at 48 kHz: three 600000-sample chunks with their seams), plus the
clean_audio wiring of convert_audio."""
import numpy as np
import pytest
import torch

from oracle import denoise as od
from rvc_amd import denoise, synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def ulps(a, ref):
    return np.abs(a - ref).max() / np.spacing(np.float32(np.abs(ref).max()))


@pytest.mark.parametrize("case", ["a", "b", "c"])
def test_denoise_matches_reference(golden, case):
    g = golden("denoise")
    sr, prop, cs, pad = g[f"{case}_meta"]
    y = g[f"{case}_y"]
    out = denoise.reduce_noise(y, int(sr), prop_decrease=float(prop), chunk_size=int(cs), padding=int(pad),
                               device=DEV)
    ref = g[f"{case}_out"]
    assert out.dtype == np.float32 and out.shape == ref.shape
    assert ulps(out, ref) <= 2.0  # both f64 end to end; rounding to f32 once


def test_denoise_30s_48k_chunked_matches_oracle():
    y = synthetic.synthetic_audio(30.0, seed=77, sr=48000).astype(np.float32)
    assert y.size > 2 * 600000  # three chunks: two seams
    out = denoise.reduce_noise(torch.from_numpy(y).to(DEV), 48000, prop_decrease=0.7).cpu().numpy()
    ref = od.reduce_noise(y, 48000, prop_decrease=0.7)
    assert ulps(out, ref) <= 2.0
    # the gate does attenuate: the output carries less energy than the input
    assert float(np.sum(out.astype(np.float64) ** 2)) < float(np.sum(y.astype(np.float64) ** 2))


@pytest.mark.parametrize("sr,prop", [(16000, 1.0), (32000, 0.0), (96000, 0.5)])
def test_denoise_rates_match_oracle(sr, prop):
    rng = np.random.default_rng(sr)
    n = int(sr * 1.3)
    t = np.arange(n) / sr
    y = (0.4 * np.sin(2 * np.pi * 330 * t) + 0.05 * rng.standard_normal(n)).astype(np.float32)
    out = denoise.reduce_noise(y, sr, prop_decrease=prop, device=DEV)
    ref = od.reduce_noise(y, sr, prop_decrease=prop)
    assert ulps(out, ref) <= 2.0
    if prop == 0.0:  # mask 1 before smoothing: only the zero-padded smoothing edges (DC / Nyquist bins) gate
        assert np.abs(out - y).max() < 0.1 * np.abs(y).max()


def test_denoise_rejects_short_and_bad_input():
    with pytest.raises(ValueError):
        denoise.reduce_noise(np.zeros(100, np.float32), 48000, chunk_size=50, padding=10, device=DEV)
    with pytest.raises(NotImplementedError):
        denoise.reduce_noise(np.zeros(48000, np.float32), 48000, stationary=True, device=DEV)


def test_convert_audio_clean_audio(tmp_path):
    from rvc_amd import audio_io
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.convert import VoiceConverterAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(32), DEV)
    rm = RMVPEAMD(synthetic.rmvpe_state_dict(33), DEV)
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(48000, "v2", seed=31), DEV)
    vc = VC(48000, Config(DEV), rmvpe=rm)
    src = str(tmp_path / "in.wav")
    audio_io.write_wav(src, synthetic.synthetic_audio(3.0, seed=12), 16000)
    cvt = VoiceConverterAMD(vc, net_g, hub, 48000, "v2")
    kw = dict(pitch=0, f0_method="rmvpe", index_rate=0.0, protect=0.33)
    vc.seed = 3
    raw = cvt.convert_audio(src, str(tmp_path / "raw.wav"), **kw)
    vc.seed = 3
    clean = cvt.convert_audio(src, str(tmp_path / "clean.wav"), clean_audio=True, clean_strength=0.6, **kw)
    assert raw is not None and clean is not None and clean.shape == raw.shape
    assert ulps(clean, od.reduce_noise(raw, 48000, prop_decrease=0.6)) <= 2.0
