"""Synthesizer.infer on the HIP path vs the reference's own outputs (golden vectors) and the oracle."""
import numpy as np
import pytest
import torch

from rvc_amd import synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rms(a, b):
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = b.detach().cpu().double().numpy() if torch.is_tensor(b) else np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.sqrt(np.mean((a - b) ** 2)))


# the TextEncoder / flow |max| switches (synth.py): the defaults, every cell on, the f32 attention without cells, and the
# noise convs as the upsampling call's source pass (off by default)
SWITCHES = {"default": {}, "cells_on": dict(TE_AMAX=True, FLOW_AMAX=True, ATTN_F16=True),
            "cells_off": dict(TE_AMAX=False, FLOW_AMAX=False, ATTN_F16=False), "fused_noise": dict(FUSED_NOISE=True)}


@pytest.mark.parametrize("sw", list(SWITCHES))
@pytest.mark.parametrize("name", ["synth_48k_v2", "synth_40k_v2", "synth_32k_v1"])
def test_synth_infer_matches_reference_golden(golden, name, sw, monkeypatch):
    from rvc_amd import synth
    from rvc_amd.synth import SynthesizerAMD
    for k, v in SWITCHES[sw].items():
        monkeypatch.setattr(synth, k, v)
    g = golden(name)
    ck = synthetic.make_synth_ckpt(int(g["sr"]), str(g["version"]), seed=int(g["seed"]))
    net = SynthesizerAMD(ck, DEV)
    T = int(g["T"])
    o, x_mask, (z, z_p, m_p, logs_p) = net.infer(
        torch.from_numpy(g["phone"]).to(DEV), torch.tensor([T], device=DEV), torch.from_numpy(g["pitch"]).to(DEV),
        torch.from_numpy(g["pitchf"]).to(DEV), torch.from_numpy(g["sid"]).to(DEV),
        z_noise=torch.from_numpy(g["z_noise"]).to(DEV), sine_noise=torch.from_numpy(g["sine_noise"]).to(DEV))
    torch.cuda.synchronize()
    # tolerance: 1e-4 RMS on the waveform (BASELINE.json north_star, fp32)
    assert rms(m_p, g["m_p"]) < 1e-5
    assert rms(logs_p, g["logs_p"]) < 1e-5
    assert rms(z_p, g["z_p"]) < 1e-5
    assert rms(z, g["z"]) < 1e-5
    assert rms(o, g["o"]) < 1e-4


def test_synth_device_noise_is_deterministic():
    from rvc_amd.synth import SynthesizerAMD
    ck = synthetic.make_synth_ckpt(48000, "v2", seed=5)
    net = SynthesizerAMD(ck, DEV)
    T = 64
    phone = torch.randn(1, T, 768, generator=torch.Generator().manual_seed(0)).to(DEV)
    pitch = torch.randint(1, 255, (1, T), generator=torch.Generator().manual_seed(1)).to(DEV)
    pitchf = (torch.rand(1, T, generator=torch.Generator().manual_seed(2)) * 400).to(DEV)
    a = net.infer(phone, torch.tensor([T]), pitch, pitchf, 0, seed=7)[0]
    b = net.infer(phone, torch.tensor([T]), pitch, pitchf, 0, seed=7)[0]
    c = net.infer(phone, torch.tensor([T]), pitch, pitchf, 0, seed=8)[0]
    assert torch.equal(a, b)
    assert not torch.equal(a, c)
    assert a.shape == (1, 1, T * 480)
    assert torch.isfinite(a).all() and float(a.abs().max()) <= 1.0
