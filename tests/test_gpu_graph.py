"""hipGraph-captured clip loop (rvc_amd.graph.ClipGraph) against the eager VC.pipeline_device: the
replay must give the eager waveform bit for bit at the same seed, fresh noise per seed, and new
input on every replay (BASELINE configs[4]: per-GPU hipGraph-captured chunk loop)."""
import numpy as np
import pytest
import torch

from rvc_amd import ops, synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def build(sr=48000, version="v2", seed=7):
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(sr, version, seed=seed), DEV)
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(seed + 1), DEV)
    vc = VC(sr, Config(DEV), rmvpe=RMVPEAMD(synthetic.rmvpe_state_dict(seed + 2), DEV))
    return vc, hub, net_g


def eager(vc, hub, net_g, audio, seed, f0_method="rmvpe", dev_seed=None):
    vc.seed = seed
    if dev_seed is None:
        return vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33, None, 0.0, f0_method).clone()
    t = torch.zeros(1, dtype=torch.int64, device=DEV)  # graph-mode draws (device dither) at seed 0 + seed
    vc.seed = 0
    t.fill_(seed)
    with ops.device_seed(t):
        return vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33, None, 0.0, f0_method).clone()


def test_clip_graph_matches_eager():
    from rvc_amd.graph import ClipGraph
    vc, hub, net_g = build()
    a1 = torch.from_numpy(synthetic.synthetic_audio(3.0, seed=1001)).to(DEV)
    a2 = torch.from_numpy(synthetic.synthetic_audio(3.0, seed=1002)).to(DEV)
    g = ClipGraph(vc, hub, net_g, 0, a1.numel())
    outs = {}
    for audio, seed in ((a1, 5), (a2, 5), (a1, 6), (a1, 5)):  # new input / new seed / back again
        got = g(audio, seed).clone()
        torch.cuda.synchronize()
        ref = eager(vc, hub, net_g, audio, seed)
        assert got.shape == ref.shape
        assert torch.equal(got, ref), float((got - ref).abs().max())
        outs[(audio.data_ptr(), seed)] = got
    vc.rmvpe.check_error()
    # the seed moves the device noise, the input moves everything
    assert not torch.equal(outs[(a1.data_ptr(), 5)], outs[(a1.data_ptr(), 6)])
    assert not torch.equal(outs[(a1.data_ptr(), 5)], outs[(a2.data_ptr(), 5)])
    assert np.isfinite(outs[(a1.data_ptr(), 5)].cpu().numpy()).all()


def test_clip_graph_crepe_device_dither():
    from rvc_amd.crepe import CrepeAMD
    from rvc_amd.graph import ClipGraph
    vc, hub, net_g = build()
    vc.crepe["tiny"] = CrepeAMD(synthetic.crepe_state_dict(1240, "tiny"), "tiny", DEV)
    a = torch.from_numpy(synthetic.synthetic_audio(2.0, seed=1003)).to(DEV)
    g = ClipGraph(vc, hub, net_g, 0, a.numel(), f0_method="crepe-tiny")
    got = g(a, 9).clone()
    torch.cuda.synchronize()
    ref = eager(vc, hub, net_g, a, 9, "crepe-tiny", dev_seed=True)
    assert torch.equal(got, ref), float((got - ref).abs().max())


def test_triangular_dither_law():
    """The device dither has scipy.stats.triang(c=0.5, loc=-20, scale=40)'s law (CREPE.py:118)."""
    from scipy import stats
    x = ops.rand_triang(torch.empty(1 << 20, device=DEV), -20.0, 20.0, 123, 0).cpu().numpy()
    assert x.min() >= -20 and x.max() <= 20
    assert abs(x.mean()) < 0.05 and abs(x.var() - 40 ** 2 / 24) < 0.5
    assert stats.kstest(x[:20000], stats.triang(c=0.5, loc=-20, scale=40).cdf).pvalue > 1e-3


def test_clip_graph_rejects_long_input():
    from rvc_amd.graph import ClipGraph
    vc, hub, net_g = build()
    with pytest.raises(ValueError):
        ClipGraph(vc, hub, net_g, 0, vc.t_max)
