"""Equal-length clips batched through RMVPE and ContentVec (VC.pipeline_device_batch, BASELINE configs[2]
chunk loop): each batched stage against the same stage run clip by clip, and the whole batched pass
against per-clip pipeline_device."""
import numpy as np
import pytest
import torch

from rvc_amd import ops, synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def models():
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(71), DEV)
    rm = RMVPEAMD(synthetic.rmvpe_state_dict(72), DEV)
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(48000, "v2", seed=73), DEV)
    return hub, rm, net_g, VC(48000, Config(DEV), rmvpe=rm)


def clips(n, secs, seed):
    return [torch.from_numpy(synthetic.synthetic_audio(secs, seed=seed + i)).to(DEV) for i in range(n)]


@pytest.mark.parametrize("B", [1, 3, 18])
def test_bigru_batched_bit_identical(models, B):
    _, rm, _, _ = models
    T = 96
    g = torch.Generator().manual_seed(B)
    gi = (torch.randn(B, 1536, T, generator=g) * 0.5).to(DEV)
    y = torch.empty(B, 512, T, device=DEV)
    gran = torch.zeros(1024 * min(B, ops.GRU_B_MAX), dtype=torch.int64, device=DEV)
    ops.bigru_batched(gi, rm.w_hh, rm.b_hh, y, gran, rm.err, B, T)
    for b in range(B):
        yb = torch.empty(512, T, device=DEV)
        ops.bigru(gi[b].contiguous(), rm.w_hh, rm.b_hh, yb, rm.gran, rm.err, T)
        assert torch.equal(y[b], yb)
    rm.check_error()


def test_contentvec_batched_matches_per_clip(models):
    hub = models[0]
    xs = clips(3, 3.0, 300)
    fb = hub.features_cf(torch.stack(xs), 12)
    for b, x in enumerate(xs):
        f1 = hub.features_cf(x, 12)
        assert fb.shape[1:] == f1.shape
        err = (fb[b] - f1).abs().max().item()
        assert err <= 2e-5 * max(1.0, f1.abs().max().item()), err


def test_rmvpe_batched_matches_per_clip(models):
    _, rm, _, vc = models
    xs = clips(3, 4.0, 400)
    xp = torch.stack([vc.filt(x, vc.t_pad)[0] for x in xs])
    mel_b = rm.mel_spectrogram_batch(xp)
    sal_b, Tp = rm.salience_batch(mel_b)
    coarse_b, pitchf_b = rm.f0_device_batch(xp)
    for b in range(3):
        mel = rm.mel_spectrogram(xp[b])
        # log-mel: the batched DFT GEMM sums in another split-K order; log(max(., 1e-5)) magnifies the
        # relative rounding of the near-cancelling bins
        assert (mel_b[b] - mel).abs().max().item() <= 2e-3
        sal, Tp1 = rm.salience(mel)
        assert Tp1 == Tp
        assert (sal_b[b] - sal).abs().max().item() <= 2e-3
        coarse, pitchf, _ = rm.f0_device(xp[b])
        same = (coarse_b[b] == coarse).float().mean().item()
        assert same >= 0.995, same
    rm.check_error()


def test_pipeline_batch_matches_per_clip(models):
    hub, rm, net_g, vc = models
    xs = clips(3, 4.0, 500)
    vc.seed = 40
    outs = vc.pipeline_device_batch(hub, net_g, 0, xs, 0, "v2", 0.33)
    for b, x in enumerate(xs):
        vc.seed = 40 + b
        ref = vc.pipeline_device(hub, net_g, 0, x, 0, "v2", 0.33)
        assert outs[b].shape == ref.shape
        rel = ((outs[b] - ref).double().pow(2).mean().sqrt() / ref.double().pow(2).mean().sqrt()).item()
        assert rel <= 1e-4, (b, rel)
    vc.check_errors()


def test_stream_bit_identical_to_per_clip(models):
    """VC.pipeline_device_stream (clip k+1's front end under clip k's synthesizer, three streams) gives every
    clip exactly the waveform of pipeline_device at seed + k: same launches on the same data."""
    hub, _, net_g, vc = models
    xs = clips(3, 5.0, 700)
    vc.seed = 40
    outs = vc.pipeline_device_stream(hub, net_g, 0, xs, 0, "v2", 0.33)
    torch.cuda.synchronize()
    assert vc.seed == 40
    for k, x in enumerate(xs):
        vc.seed = 40 + k
        ref = vc.pipeline_device(hub, net_g, 0, x, 0, "v2", 0.33)
        assert outs[k].shape == ref.shape
        assert torch.equal(outs[k], ref), (k, (outs[k] - ref).abs().max().item())
    vc.seed = 0
    vc.check_errors()


def test_batched_stream_bit_identical_to_batch(models):
    """pipeline_device_stream(batch=3) over 5 clips = pipeline_device_batch of groups [0:3], [3:5] (same
    batched front-end launches, seeds self.seed + k)."""
    hub, _, net_g, vc = models
    xs = clips(5, 4.0, 800)
    vc.seed = 7
    outs = vc.pipeline_device_stream(hub, net_g, 0, xs, 0, "v2", 0.33, batch=3)
    torch.cuda.synchronize()
    ref = vc.pipeline_device_batch(hub, net_g, 0, xs[:3], 0, "v2", 0.33)
    vc.seed = 10
    ref += vc.pipeline_device_batch(hub, net_g, 0, xs[3:], 0, "v2", 0.33)
    vc.seed = 0
    torch.cuda.synchronize()
    assert len(outs) == 5
    for k in range(5):
        assert torch.equal(outs[k], ref[k]), (k, (outs[k] - ref[k]).abs().max().item())
    vc.check_errors()
