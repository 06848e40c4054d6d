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


@pytest.mark.parametrize("f64", [False, True, "f32rec"])
@pytest.mark.parametrize("B", [1, 3, 18])
def test_bigru_batched_bit_identical(models, B, f64):
    """B recurrences side by side (two launches at B = 18) equal each sequence's own launch, in the f32 form
    (rmvpe.hip) and the f64 interface (rmvpe64.hip) with its recurrence in f64 or in f32 (the default), and the f64
    interface matches torch's f64 GRU on the host: to 1e-12 all-f64, to 2e-6 with the f32 recurrence."""
    _, rm, _, _ = models
    lib = ops._lib.load()
    lib.rvc_bigru64_set_f32(1 if f64 == "f32rec" else 0)
    try:
        _bigru_case(rm, B, f64)
    finally:
        lib.rvc_bigru64_set_f32(-1)


def _bigru_case(rm, B, f64):
    T = 96
    dt = torch.float64 if f64 else torch.float32
    g = torch.Generator().manual_seed(B)
    gi = (torch.randn(B, 1536, T, generator=g, dtype=torch.float64) * 0.5).to(dt).to(DEV)
    whh = (torch.randn(2, 768, 256, generator=g, dtype=torch.float64) * 0.06).to(dt).to(DEV)
    bhh = (torch.randn(2, 768, generator=g, dtype=torch.float64) * 0.1).to(dt).to(DEV)
    y = torch.empty(B, 512, T, device=DEV, dtype=dt)
    words = ops.GRU64_GRAN if f64 else 1024
    gran = torch.zeros(words * min(B, ops.GRU_B_MAX), dtype=torch.int64, device=DEV)
    (ops.bigru64_batched if f64 else ops.bigru_batched)(gi, whh, bhh, y, gran, rm.err, B, T)
    for b in range(B):
        yb = torch.empty(1, 512, T, device=DEV, dtype=dt)
        g1 = torch.zeros(words, dtype=torch.int64, device=DEV)
        if f64:
            ops.bigru64_batched(gi[b:b + 1].contiguous(), whh, bhh, yb, g1, rm.err, 1, T)
        else:
            ops.bigru(gi[b].contiguous(), whh, bhh, yb[0], g1, rm.err, T)
        assert torch.equal(y[b], yb[0])
    rm.check_error()
    if f64:  # torch's own f64 GRU (what oracle.rmvpe.bigru_torch runs), fed the same gi through an identity W_ih
        x = gi[0].cpu().t()  # [T][1536]
        gru = torch.nn.GRU(1536, 256, bidirectional=True, batch_first=True).double()
        with torch.no_grad():
            for d, sfx in enumerate(("", "_reverse")):
                eye = torch.zeros(768, 1536, dtype=torch.float64)
                eye[:, d * 768:(d + 1) * 768] = torch.eye(768, dtype=torch.float64)
                getattr(gru, "weight_ih_l0" + sfx).copy_(eye)
                getattr(gru, "bias_ih_l0" + sfx).zero_()
                getattr(gru, "weight_hh_l0" + sfx).copy_(whh[d].cpu())
                getattr(gru, "bias_hh_l0" + sfx).copy_(bhh[d].cpu())
            want = gru(x.unsqueeze(0))[0][0].t()  # [512][T]
        assert (y[0].cpu() - want).abs().max().item() < (2e-6 if f64 == "f32rec" else 1e-12)


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
    import f0check
    _, _, f0_b, _ = rm.f0_device_batch(xp, want_f0=True, want_salience=True)
    for b in range(3):
        mel = rm.mel_spectrogram(xp[b])
        # the |STFT| is per frame (f64 FFT) in both; the mel GEMM may sum in another split-K order
        assert (mel_b[b] - mel).abs().max().item() <= 1e-4
        sal, Tp1 = rm.salience(mel)
        assert Tp1 == Tp
        assert (sal_b[b] - sal).abs().max().item() <= 2e-3
        coarse, pitchf, _ = rm.f0_device(xp[b])
        # the f0-decision rule of tests/f0check.py for the batched path: its salience within the reference's own
        # f32 noise of the exact (f64) model, and a decision different from the exact model's -- hence from the
        # per-clip path's, also checked -- only where the exact margin is below the reference's decision noise
        F = mel.shape[-1]
        audio = xs[b].cpu().numpy()
        sd_b = sal_b[b, :, :F].t().cpu().numpy().astype(np.float64)
        sd_1 = sal[:, :F].t().cpu().numpy().astype(np.float64)
        _, _, rep_b = f0check.check(None, synthetic.rmvpe_state_dict(72), audio,
                                    device=(sd_b, f0_b[b].cpu().numpy()), exact=rm.f64)
        _, _, rep_1 = f0check.check(None, synthetic.rmvpe_state_dict(72), audio, device=(sd_1, None), exact=rm.f64)
        differ = np.flatnonzero((coarse_b[b] != coarse).cpu().numpy())
        allowed = set(rep_b["flips_vs_exact"]) | set(rep_1["flips_vs_exact"])
        for t in differ:  # the coarse quantiser of an equal decision may still round a 1e-6 pitch change
            if t not in allowed:
                assert abs(pitchf_b[b, t].item() - pitchf[t].item()) <= 1e-3 * max(1.0, pitchf[t].item()), t
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


def test_stream_host_out_30s_bit_identical_to_per_call(models):
    """The bench's form of the stream -- 30 s clips, each output copied to pinned host memory on the synthesizer's
    stream (host_out) -- against vc.pipeline_device per clip (the per-call form the headline parity test runs):
    every clip's host copy equals the per-call waveform bit for bit."""
    hub, _, net_g, vc = models
    xs = clips(2, 30.0, 900)
    vc.seed = 21
    host = [torch.empty(30 * 48000 + 48000, dtype=torch.float32).pin_memory() for _ in xs]
    outs = vc.pipeline_device_stream(hub, net_g, 0, xs, 0, "v2", 0.33, host_out=host)
    torch.cuda.synchronize()
    for k, x in enumerate(xs):
        vc.seed = 21 + k
        ref = vc.pipeline_device(hub, net_g, 0, x, 0, "v2", 0.33).cpu()
        n = ref.numel()
        assert outs[k].numel() == n and n <= host[k].numel()
        assert torch.equal(host[k][:n], ref), (k, (host[k][:n] - ref).abs().max().item())
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


@pytest.mark.parametrize("C,K,dil", [(32, 3, 5), (64, 7, 3), (64, 11, 1)])
def test_resblock_pair_batched_bit_identical(models, C, K, dil):
    """The fused ResBlock pair over [B][C][L]: each clip bit-identical to its own launch (per-tile scales and
    summation order do not depend on the batch)."""
    g = torch.Generator().manual_seed(C + K)
    c1 = ops.Conv(torch.randn(C, C, K, generator=g) * 0.1, torch.randn(C, generator=g) * 0.1, device=DEV)
    c2 = ops.Conv(torch.randn(C, C, K, generator=g) * 0.1, torch.randn(C, generator=g) * 0.1, device=DEV)
    if not ops.resblock_fusable(c1, c2, dil):
        pytest.skip("fused ResBlock off")
    B, L = 3, 5000
    x = torch.randn(B, C, L, generator=g).to(DEV)
    y0 = torch.randn(B, C, L, generator=g).to(DEV)
    for acc in (False, True):
        y = y0.clone()
        ops.resblock_pair(x, y, c1, c2, dil, 0.1, accumulate=acc)
        for b in range(B):
            yb = y0[b].clone()
            ops.resblock_pair(x[b].contiguous(), yb, c1, c2, dil, 0.1, accumulate=acc)
            assert torch.equal(y[b], yb), (acc, b, (y[b] - yb).abs().max().item())


def test_synth_batched_matches_per_clip(models):
    """SynthesizerAMD.prior_batch + decode_batch (TextEncoder, prior, flow^-1, NSF generator as B-clip
    launches) against infer_cf per clip at the same seeds: equal up to the batched launches' split-K /
    split-KV order."""
    net_g = models[2]
    B, T = 3, 400
    g = torch.Generator().manual_seed(5)
    phone = (torch.randn(B, net_g.emb_dim, T, generator=g)).to(DEV)
    pitch = torch.randint(1, 255, (B, T), generator=g).to(DEV)
    nsff0 = (100 + 200 * torch.rand(B, T, generator=g)).to(DEV)
    nsff0[:, 50:80] = 0  # unvoiced run
    seeds = [11, 12, 13]
    z, _, stats, gc = net_g.prior_batch(phone, pitch, 0, None, seeds)
    o = net_g.decode_batch(z, nsff0, gc, None, seeds)
    for b in range(B):
        o1, z1, _, st1 = net_g.infer_cf(phone[b].contiguous(), pitch[b].contiguous(), nsff0[b].contiguous(), 0,
                                        seed=seeds[b])
        assert (stats[b] - st1).abs().max().item() <= 1e-5 * max(1.0, st1.abs().max().item())
        assert (z[b] - z1).abs().max().item() <= 1e-5 * max(1.0, z1.abs().max().item())
        rel = ((o[b] - o1).double().pow(2).mean().sqrt() / o1.double().pow(2).mean().sqrt()).item()
        assert rel <= 1e-5, (b, rel)
