"""End-to-end VC.pipeline on the HIP path vs the reference's own outputs (golden vectors)."""
import types

import numpy as np
import pytest
import torch

import f0check
from rvc_amd import synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def build(sr, version, seed):
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(sr, version, seed=seed), DEV)
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(seed + 1), DEV)
    vc = VC(sr, Config(DEV), rmvpe=RMVPEAMD(synthetic.rmvpe_state_dict(seed + 2), DEV))
    return vc, hub, net_g


class Pbar:
    n = 0

    def update(self, k):
        self.n += k


@pytest.mark.parametrize("name", ["pipeline_48k_v2", "pipeline_32k_v1", "pipeline_48k_v2_opts"])
def test_pipeline_matches_reference_golden(golden, name, tmp_path):
    g = golden(name)
    sr, version, seed = int(g["sr"]), str(g["version"]), int(g["seed"])
    vc, hub, net_g = build(sr, version, seed)

    def noise(seg, kind, shape):
        a = torch.from_numpy(g[f"{'z' if kind == 'z' else 'sine'}_noise_{seg}"]).to(DEV)
        assert tuple(a.shape) == tuple(shape)
        return a

    vc.noise_fn = noise
    pb = Pbar()
    f0_file = None
    if "f0_lines" in g:  # the reference reads f0_file.name (convert.py:427)
        path = tmp_path / "f0.txt"
        path.write_text("\n".join(str(x) for x in g["f0_lines"]) + "\n")
        f0_file = types.SimpleNamespace(name=str(path))
    out = vc.pipeline(model=hub, net_g=net_g, sid=0, audio=g["audio"].copy(), pitch=float(g["pitch"]),
                      f0_method="rmvpe", file_index="", index_rate=0.0, pitch_guidance=1, filter_radius=3,
                      volume_envelope=float(g.get("volume_envelope", 1)), version=version,
                      protect=float(g["protect"]), hop_length=64, f0_autotune="f0_autotune_strength" in g,
                      f0_autotune_strength=float(g.get("f0_autotune_strength", 1)), suffix=".pth",
                      embed_suffix=".pt", f0_file=f0_file, pbar=pb)
    vc.rmvpe.check_error()
    assert out.dtype == np.float32 and out.shape == g["out"].shape
    err = float(np.sqrt(np.mean((out.astype(np.float64) - g["out"]) ** 2)))
    # BASELINE.json north_star tolerance: waveform within 1e-4 RMS of the reference CPU path (fp32)
    assert err < 1e-4, err
    assert pb.n > 0


def test_long_input_segments_vs_oracle():
    """45 s input (> x_max = 41 s): quiet-point segmentation + multi-segment stitching vs the CPU oracle."""
    from oracle import contentvec as ocv
    from oracle import pipeline as opl
    from oracle import rmvpe as orm
    from oracle import synth as osy
    from rvc_amd import melbasis
    sr, version, seed = 32000, "v2", 61
    vc, hub, net_g = build(sr, version, seed)
    audio = synthetic.synthetic_audio(45.0, seed=9)
    noises = {}

    def noise(seg, kind, shape):
        key = (seg, kind)
        if key not in noises:
            noises[key] = torch.randn(*shape, generator=torch.Generator().manual_seed(100 * seg + len(kind)))
        assert tuple(noises[key].shape) == tuple(shape)
        return noises[key]

    vc.noise_fn = lambda s, k, sh: noise(s, k, sh).to(DEV)
    assert len(vc.segment_points(opl.signal.filtfilt(opl.BH, opl.AH, audio))) == 1
    out = vc.pipeline(hub, net_g, 0, audio.copy(), 0, "rmvpe", "", 0.0, 1, 3, 1, version, 0.33, 64, False, 1, ".pth",
                      ".pt")
    ck = synthetic.make_synth_ckpt(sr, version, seed=seed)
    torch.set_num_threads(16)
    Wc, Ws = ocv.load_weights(synthetic.make_contentvec_ckpt(seed + 1)), osy.load_weights(ck["weight"])
    Wr = orm.load_weights(synthetic.rmvpe_state_dict(seed + 2))
    mb = torch.from_numpy(melbasis.mel_filterbank())
    # f0 decisions vs the exact model (tests/f0check.py), then the waveform within 1e-4 RMS of the oracle
    f0check.assert_pipeline(vc, out, synthetic.rmvpe_state_dict(seed + 2), audio, lambda f0: opl.pipeline(
        Wc, Ws, Wr, mb, ck["config"], 0, audio, 0.0, version, 0.33, noise, f0_track=f0))


def test_change_rms_matches_reference(golden):
    """change_rms (convert.py:150-152) on the device vs the reference's output (f0_opts golden)."""
    from rvc_amd import ops
    g = golden("f0_opts")
    src64 = torch.from_numpy(g["rms_src"]).to(DEV)
    out = torch.from_numpy(g["rms_tgt"]).to(DEV)
    ops.change_rms(None, src64, out, 8000, 0.35)
    np.testing.assert_allclose(out.cpu().numpy(), g["rms_out"], rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_f0_post_autotune_override(golden, dtype):
    """The decode kernels' autotune + shift + f0-file steps (rvc_f0_post) vs the reference: the f64 RMVPE
    path through rmvpe_decode on a one-hot salience, the f32 CREPE path through crepe_smooth_coarse."""
    import ctypes
    from rvc_amd import _lib, ops
    from rvc_amd.pipeline import f0_override
    from oracle import pipeline as opl
    g = golden("f0_opts")
    c = opl.Consts(48000)
    rep, off = f0_override(g["inp_f0"], 1)
    if dtype == "f64":
        # a salience with one bin (i) above threshold decodes to f0 = 10 * 2^((20 i + 1997.379...) / 1200)
        T = 600
        rng = np.random.default_rng(5)
        bins = rng.integers(0, 360, T)
        sal = np.zeros((360, T), np.float32)
        sal[bins, np.arange(T)] = 0.9
        sal[:, ::13] = 0.0  # unvoiced frames (autotune moves them to 49 * strength)
        post = ops.F0Post(0.6, rep, off, DEV)
        coarse = torch.empty(T, dtype=torch.int64, device=DEV)
        pitchf = torch.empty(T, device=DEV)
        f0 = torch.empty(T, dtype=torch.float64, device=DEV)
        ops.rmvpe_decode(torch.from_numpy(sal).to(DEV), T, T, 0.03, 2 ** (3 / 12), f0, coarse, pitchf, post)
        raw = np.where(sal.max(0) > 0.03, 10 * 2 ** ((20 * bins + 1997.3794084376191) / 1200), 0.0)
        raw[raw == 10] = 0
        ref_c, ref_f0 = opl.coarse_f0(raw, 3, c, 0.6, g["inp_f0"])
        np.testing.assert_allclose(f0.cpu().numpy(), ref_f0, rtol=1e-12)
    else:
        track = g["f32"][:600].copy()
        T = track.size
        post = ops.F0Post(0.75, rep, off, DEV)
        # pd = 1 everywhere; mean-3 smoothing is undone by feeding a constant-run track (each value x3)
        f0r = np.repeat(track, 3)
        pd = np.ones_like(f0r)
        T3 = f0r.size
        coarse = torch.empty(T3, dtype=torch.int64, device=DEV)
        pitchf = torch.empty(T3, device=DEV)
        lib = _lib.load()
        st = post.struct(T3)
        f0r_d, pd_d = torch.from_numpy(f0r).to(DEV), torch.from_numpy(pd).to(DEV)  # held across the launch
        _lib.check(lib.rvc_crepe_smooth_coarse(ops._p(f0r_d), ops._p(pd_d), T3, ctypes.c_float(2 ** (3 / 12)),
                                               c.f0_mel_min, c.f0_mel_max, ctypes.byref(st), ops._p(coarse),
                                               ops._p(pitchf), ops._stream()), "crepe_smooth_coarse")
        sm = np.convolve(f0r, np.ones(3, np.float32), "same").astype(np.float32)
        cnt = np.full(T3, 3.0, np.float32)
        cnt[0] = cnt[-1] = 2
        sm = (sm / cnt).astype(np.float32)
        at = opl.autotune_f0(sm, 0.75)
        ref_f0 = at * np.float32(2 ** (3 / 12))
        ref_f0[off: off + rep.size] = rep[:max(0, min(rep.size, T3 - off))]
        # interior frames of each run are exact copies; compare those (edges go through the mean)
        inner = np.arange(T3) % 3 == 1
        np.testing.assert_allclose(pitchf.cpu().numpy()[inner], ref_f0[inner], rtol=1e-6)
        return
    np.testing.assert_array_equal(coarse.cpu().numpy(), ref_c)
    np.testing.assert_array_equal(pitchf.cpu().numpy(), ref_f0.astype(np.float32))


@pytest.mark.parametrize("seconds", [41.5, 95.0, 200.0])
def test_quiet_points_device_equals_reference_search(seconds):
    """ops.quiet_points (pipeline.hip) vs the reference's numpy search (VC.segment_points, convert.py:404-412)
    on a filtered f64 signal with digital-silence runs (exact |sum| = 0 ties: the first index wins) and a
    non-silent stretch: identical quiet points."""
    from rvc_amd import ops
    from rvc_amd.pipeline import VC, Config
    vc = VC(48000, Config(DEV))
    x = synthetic.synthetic_audio(seconds, seed=3).astype(np.float64)
    x[int(50.0 * 16000): int(52.5 * 16000)] = 0.0  # a silence run inside the second search window
    x64 = vc.filt(torch.from_numpy(x.astype(np.float32)).to(DEV), 0, want_f64=True)[1]
    want = vc.segment_points(x64.cpu().numpy())
    got = ops.quiet_points(x64, vc.window, vc.t_center, vc.t_query, vc.t_max)
    assert got == [int(t) for t in want], (got, want)
    assert len(got) == (len(x) - 1) // vc.t_center
