"""CREPE f0 on the device (crepe.hip + the conv engines) vs the reference's golden outputs
(tests/golden/crepe.npz: the reference's Crepe network / per-batch decode with recorded dither) and
vs the CPU oracle inside VC.pipeline.  librosa's Viterbi is restated (parity unpinned, see oracle/crepe.py)."""
import numpy as np
import pytest
import torch

from rvc_amd import synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def crepe_golden(golden):
    from rvc_amd.crepe import CrepeAMD
    g = golden("crepe")
    m = CrepeAMD(synthetic.crepe_state_dict(int(g["seed"])), "full", DEV)
    m.dither_fn = lambda T: g["dither"][:T]
    return m, g


def test_crepe_network_matches_reference(crepe_golden):
    m, g = crepe_golden
    tr = {}
    m.f0_device(torch.from_numpy(g["audio"].astype(np.float32)).to(DEV), 0.0, trace=tr)
    err = np.abs(tr["probs"] - g["probs"])
    assert err.max() < 2e-5, err.max()


def test_crepe_f0_matches_reference(crepe_golden):
    """f0 through get_f0 (coarse + pitchf) vs the reference's get_f0_crepe output pushed through the
    oracle's restatement of get_f0 (convert.py:311-323)."""
    from oracle.pipeline import Consts, coarse_f0
    m, g = crepe_golden
    coarse, pitchf = m.f0_device(torch.from_numpy(g["audio"].astype(np.float32)).to(DEV), 2.0)
    ref_c, ref_f = coarse_f0(g["f0"].copy(), 2.0, Consts(48000))
    pf = pitchf.cpu().numpy()
    np.testing.assert_allclose(pf, ref_f, rtol=1e-4, atol=1e-3)
    # the decode is discrete: allow the rare frame where f32 rounding moves a coarse bin by one
    c = coarse.cpu().numpy()
    assert np.mean(c == ref_c) > 0.99 and np.max(np.abs(c - ref_c)) <= 1


@pytest.mark.parametrize("capacity", ["tiny", "full"])
def test_pipeline_crepe_vs_oracle(capacity):
    from oracle import contentvec as ocv
    from oracle import pipeline as opl
    from oracle import rmvpe as orm
    from oracle import synth as osy
    from rvc_amd import melbasis
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.crepe import CrepeAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.synth import SynthesizerAMD
    sr, version, seed = 48000, "v2", 91
    csd = synthetic.crepe_state_dict(seed + 5, capacity)
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(sr, version, seed=seed), DEV)
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(seed + 1), DEV)
    cm = CrepeAMD(csd, capacity, DEV)
    vc = VC(sr, Config(DEV), crepe={capacity: cm})
    audio = synthetic.synthetic_audio(2.5, seed=8)
    rng = np.random.default_rng(3)
    dither = rng.triangular(-20, 0, 20, size=10000)
    cm.dither_fn = lambda T: dither[:T]
    noises = {}

    def noise(seg, kind, shape):
        if (seg, kind) not in noises:
            noises[(seg, kind)] = torch.randn(*shape, generator=torch.Generator().manual_seed(7 * seg + len(kind)))
        return noises[(seg, kind)]

    vc.noise_fn = lambda s, k, sh: noise(s, k, sh).to(DEV)
    out = vc.pipeline(hub, net_g, 0, audio.copy(), 0, f"crepe-{capacity}", "", 0.0, 1, 3, 1, version, 0.33, 64, False,
                      1, ".pth", ".pt")
    ck = synthetic.make_synth_ckpt(sr, version, seed=seed)
    torch.set_num_threads(16)
    ref = opl.pipeline(ocv.load_weights(synthetic.make_contentvec_ckpt(seed + 1)), osy.load_weights(ck["weight"]),
                       None, torch.from_numpy(melbasis.mel_filterbank()), ck["config"], 0, audio, 0.0, version, 0.33,
                       noise, crepe=(csd, capacity, dither))
    assert out.shape == ref.shape
    err = float(np.sqrt(np.mean((out.astype(np.float64) - ref) ** 2)))
    assert err < 1e-4, err
