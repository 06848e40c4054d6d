"""pm f0 on the device (csrc/pm.hip: Praat's To Pitch (ac) as VC.get_f0_pm calls it, convert.py:206-213)
against the f64 restatement oracle/pm.py, and BASELINE configs[0] (32k v1, pm f0, no index, one 5 s clip)
through VC.pipeline against the oracle pipeline.  Parity against Praat itself is unpinned (no parselmouth)."""
import numpy as np
import pytest
import torch

from rvc_amd import synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def vibrato(seconds=1.5, f=150.0, depth=0.1, rate=1.5, lead=0.5, tail=0.25, sr=16000):
    t = np.arange(int(seconds * sr)) / sr
    ph = 2 * np.pi * np.cumsum(f * (1 + depth * np.sin(2 * np.pi * rate * t))) / sr
    x = 0.5 * np.sin(ph) + 0.2 * np.sin(2 * ph) + 0.1 * np.sin(3 * ph)
    x = np.concatenate([np.zeros(int(lead * sr)), x, np.zeros(int(tail * sr))])
    return x + 1e-4 * np.random.default_rng(0).standard_normal(len(x))


def signals():
    x1 = vibrato()
    x2 = synthetic.synthetic_audio(3.0, seed=31).astype(np.float64)
    x3 = 0.3 * np.random.default_rng(5).standard_normal(16000)  # noise: mostly voiceless
    x4 = np.zeros(8000)  # no global peak: all voiceless
    return {"vibrato": x1, "speechlike": x2, "noise": x3, "silence": x4}


@pytest.mark.parametrize("name", ["vibrato", "speechlike", "noise", "silence"])
def test_pm_device_matches_oracle(name):
    from oracle import pm as opm
    from rvc_amd.pm import PitchPM
    x = signals()[name]
    ref = opm.to_pitch_ac(x)
    got = PitchPM(DEV).to_pitch_ac(torch.from_numpy(x).to(DEV)).cpu().numpy()
    assert got.shape == ref.shape
    same_v = (got > 0) == (ref > 0)
    assert same_v.mean() >= 0.99, (name, int((~same_v).sum()))
    both = (got > 0) & (ref > 0)
    if both.any():
        rel = np.abs(got[both] / ref[both] - 1)
        assert np.mean(rel < 1e-6) >= 0.99, (name, float(rel.max()))
    if name == "silence":
        assert not got.any()


def test_pipeline_cfg1_pm_32k_v1_vs_oracle():
    """BASELINE configs[0]: 32k v1, pm f0, no index, one 5 s clip -- VC.pipeline on the device against the
    oracle pipeline with the same noise; f0 decisions first (pitchf), then the waveform (<= 1e-4 RMS)."""
    from oracle import contentvec as ocv
    from oracle import pipeline as opl
    from oracle import pm as opm
    from oracle import synth as osy
    from rvc_amd import melbasis
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.synth import SynthesizerAMD
    sr, version, seed = 32000, "v1", 141
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(sr, version, seed=seed), DEV)
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(seed + 1), DEV)
    vc = VC(sr, Config(DEV))
    audio = synthetic.synthetic_audio(5.0, seed=9)
    noises = {}

    def noise(seg, kind, shape):
        if (seg, kind) not in noises:
            noises[(seg, kind)] = torch.randn(*shape, generator=torch.Generator().manual_seed(11 * seg + len(kind)))
        return noises[(seg, kind)]

    vc.noise_fn = lambda s, k, sh: noise(s, k, sh).to(DEV)
    out = vc.pipeline(hub, net_g, 0, audio.copy(), 0, "pm", "", 0.0, 1, 3, 1, version, 0.33, 64, False, 1, ".pth",
                      ".pt")
    # the f0 decisions: device pitch track vs get_f0_pm on the same f64 filtered, padded signal
    from scipy import signal
    x64 = np.pad(signal.filtfilt(opl.BH, opl.AH, audio), (16000, 16000), mode="reflect")
    p_len = len(x64) // 160
    ref_f0 = opm.get_f0_pm(x64, p_len)
    xp, xp64 = vc.filt(torch.from_numpy(audio.astype(np.float32)).to(DEV), vc.t_pad, want_f64=True)
    _, pitchf = vc.f0_device(xp, 0, "pm", xp64=xp64)
    got_f0 = pitchf.cpu().numpy().astype(np.float64)
    assert got_f0.shape == ref_f0.shape
    assert np.mean((got_f0 > 0) == (ref_f0 > 0)) >= 0.99
    ck = synthetic.make_synth_ckpt(sr, version, seed=seed)
    ref = opl.pipeline(ocv.load_weights(synthetic.make_contentvec_ckpt(seed + 1)), osy.load_weights(ck["weight"]),
                       None, torch.from_numpy(melbasis.mel_filterbank()), ck["config"], 0, audio, 0.0, version, 0.33,
                       noise, pm=True)
    assert out.shape == ref.shape
    err = float(np.sqrt(np.mean((out.astype(np.float64) - ref) ** 2)))
    assert err < 1e-4, err


def test_pm_stream_bit_identical_to_per_clip():
    """pm f0 inside the clip stream (front end on its own streams) = pipeline_device per clip."""
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.synth import SynthesizerAMD
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(32000, "v1", seed=151), DEV)
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(152), DEV)
    vc = VC(32000, Config(DEV))
    xs = [torch.from_numpy(synthetic.synthetic_audio(3.0, seed=60 + i)).to(DEV) for i in range(2)]
    vc.seed = 3
    outs = vc.pipeline_device_stream(hub, net_g, 0, xs, 0, "v1", 0.33, f0_method="pm")
    torch.cuda.synchronize()
    for k, x in enumerate(xs):
        vc.seed = 3 + k
        ref = vc.pipeline_device(hub, net_g, 0, x, 0, "v1", 0.33, f0_method="pm")
        assert torch.equal(outs[k], ref)
