"""The model-level C ABI (rvc_ctx / rvc_load_synth / rvc_synth_infer, csrc/rvc_model.cpp) on the device:
against the reference's own Synthesizer.infer outputs (golden vectors, fp16 weight-norm checkpoints folded by
the library) and bit-for-bit against the Python launch sequence (SynthesizerAMD) on the same fp32 weights."""
import numpy as np
import pytest
import torch

from rvc_amd import ops, synthetic
from rvc_amd.native import NativeSynth
from rvc_amd.synth import SynthesizerAMD, fold_weight_norm

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rms(a, b):
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = b.detach().cpu().double().numpy() if torch.is_tensor(b) else np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.sqrt(np.mean((a - b) ** 2)))


def inputs(T, E=768, seed=0, B=1):
    g = torch.Generator().manual_seed(seed)
    phone = torch.randn(B, T, E, generator=g).to(DEV)
    pitch = torch.randint(1, 255, (B, T), generator=g).to(DEV)
    pitchf = (torch.rand(B, T, generator=g) * 400).to(DEV)
    return phone, pitch, pitchf


@pytest.mark.parametrize("name", ["synth_48k_v2", "synth_40k_v2", "synth_32k_v1"])
def test_native_synth_matches_reference_golden(golden, name):
    g = golden(name)
    ck = synthetic.make_synth_ckpt(int(g["sr"]), str(g["version"]), seed=int(g["seed"]))
    net = NativeSynth(ck, DEV)  # fp16 weight_g / weight_v pairs: folded by rvc_load_synth
    T = int(g["T"])
    o = net.infer(torch.from_numpy(g["phone"]).to(DEV), torch.tensor([T]), torch.from_numpy(g["pitch"]).to(DEV),
                  torch.from_numpy(g["pitchf"]).to(DEV), torch.from_numpy(g["sid"]),
                  z_noise=torch.from_numpy(g["z_noise"]).to(DEV), sine_noise=torch.from_numpy(g["sine_noise"]).to(DEV))[0]
    torch.cuda.synchronize()
    # tolerance: 1e-4 RMS on the waveform (BASELINE.json north_star, fp32)
    assert o.shape == g["o"].shape
    assert rms(o, g["o"]) < 1e-4


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_native_synth_bit_identical_to_python_sequence(precision):
    ck = synthetic.make_synth_ckpt(48000, "v2", seed=11)
    py = SynthesizerAMD(ck, DEV)
    nat = NativeSynth(ck, DEV, weights=fold_weight_norm(ck["weight"]), precision=precision)
    T = 300  # 144000 samples: every generator stage, fused 32/64-channel pairs included
    phone, pitch, pitchf = inputs(T)
    with ops.precision(precision):
        a = py.infer(phone, torch.tensor([T]), pitch, pitchf, 0, seed=3)[0]
    b = nat.infer(phone, torch.tensor([T]), pitch, pitchf, 0, seed=3)[0]
    torch.cuda.synchronize()
    assert a.shape == b.shape == (1, 1, T * 480)
    assert torch.equal(a, b), rms(a, b)
    # injected noise takes the same route
    zn = torch.randn(1, 192, T, generator=torch.Generator().manual_seed(5)).to(DEV)
    sn = torch.randn(1, T * 480, 1, generator=torch.Generator().manual_seed(6)).to(DEV)
    with ops.precision(precision):
        a = py.infer(phone, torch.tensor([T]), pitch, pitchf, 0, z_noise=zn, sine_noise=sn)[0]
    b = nat.infer(phone, torch.tensor([T]), pitch, pitchf, 0, z_noise=zn, sine_noise=sn)[0]
    assert torch.equal(a, b), rms(a, b)


def test_native_synth_batch_and_scratch_growth():
    ck = synthetic.make_synth_ckpt(40000, "v2", seed=12)
    nat = NativeSynth(ck, DEV)
    T = 96
    phone, pitch, pitchf = inputs(T, B=2, seed=1)
    sid = torch.tensor([0, 0])
    both = nat.infer(phone, torch.tensor([T, T]), pitch, pitchf, sid, seed=9)[0]
    one0 = nat.infer(phone[:1], torch.tensor([T]), pitch[:1], pitchf[:1], 0, seed=9)[0]
    one1 = nat.infer(phone[1:], torch.tensor([T]), pitch[1:], pitchf[1:], 0, seed=10)[0]  # sequence b draws seed + b
    assert torch.equal(both[0], one0[0]) and torch.equal(both[1], one1[0])
    # a longer call grows the scratch; the short call after it is unchanged
    pl, ql, fl = inputs(700, seed=2)
    long = nat.infer(pl, torch.tensor([700]), ql, fl, 0, seed=9)[0]
    again = nat.infer(phone[:1], torch.tensor([T]), pitch[:1], pitchf[:1], 0, seed=9)[0]
    torch.cuda.synchronize()
    assert torch.isfinite(long).all() and long.shape == (1, 1, 700 * 400)
    assert torch.equal(again, one0)


def test_native_synth_errors():
    ck = synthetic.make_synth_ckpt(48000, "v2", seed=13)
    nat = NativeSynth(ck, DEV)
    T = 16
    phone, pitch, pitchf = inputs(T)
    with pytest.raises(RuntimeError, match="sid"):
        nat.infer(phone, torch.tensor([T]), pitch, pitchf, 500)  # the synthetic ckpt has 109 speakers
    bad = dict(ck["weight"])
    del bad["dec.m_source.l_linear.bias"]
    with pytest.raises(RuntimeError, match="dec.m_source.l_linear.bias"):
        NativeSynth(ck, DEV, weights=bad)


# ------------------------------------------------------------------ ContentVec / RMVPE through the model-level ABI
def test_native_contentvec_matches_golden_and_python(golden):
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.native import NativeContentVec
    g = golden("contentvec")
    ck = synthetic.make_contentvec_ckpt(int(g["seed"]))
    nat, py = NativeContentVec(ck, DEV), ContentVecAMD(ck, DEV)
    src = torch.from_numpy(g["audio"]).view(1, -1).to(DEV)
    x2 = nat.forward(src, 12)
    x1 = nat.forward(src, 9, final_proj=True)
    torch.cuda.synchronize()
    assert rms(x2, g["feats_v2"]) < 1e-4  # the reference's own extract_features output
    assert rms(x1, g["feats_v1"]) < 1e-4
    # same launches as the Python model: bit-identical on the same folded pos_conv weight (odd T_f, 6.3 s);
    # the native weight-norm fold (f64 norm) and torch's (f32) differ in the last bits only
    wav = torch.from_numpy(synthetic.synthetic_audio(6.3, seed=77)).float().to(DEV)
    ref = py.features_cf(wav, 12).t().unsqueeze(0)
    assert rms(nat.forward(wav, 12), ref.cpu().numpy()) < 1e-5
    sd = dict(ck["model"])
    p = "encoder.pos_conv.0.weight"
    sd[p] = torch._weight_norm(sd.pop(p + "_v").float(), sd.pop(p + "_g").float(), 2)
    nat = NativeContentVec(ck, DEV, weights=sd)
    got = nat.forward(wav, 12)
    assert got.shape == ref.shape and torch.equal(got, ref)
    ref1 = py.final_proj(py.extract_features(wav.view(1, -1), output_layer=9)[0])
    assert torch.equal(nat.forward(wav, 9, final_proj=True), ref1)
    # B sequences = B single calls
    wb = torch.stack([wav, wav.flip(0)])
    both = nat.forward(wb, 12)
    assert torch.equal(both[0], got[0]) and torch.equal(both[1], nat.forward(wav.flip(0), 12)[0])


def test_native_rmvpe_matches_golden_and_python(golden):
    from rvc_amd import melbasis
    from rvc_amd.native import NativeRMVPE
    from rvc_amd.rmvpe import RMVPEAMD
    g = golden("rmvpe")
    sd = synthetic.rmvpe_state_dict(int(g["seed"]))
    py = RMVPEAMD(sd, DEV)
    nat = NativeRMVPE(sd, DEV, window=torch.hann_window(1024), mel_basis=melbasis.mel_filterbank(16000, 1024, 128, 30, 8000))
    f0 = nat.infer_from_audio(g["audio"], thred=0.03)
    assert f0.shape == g["f0"].shape and np.max(np.abs(f0 - g["f0"])) < 1e-2  # test_gpu_rmvpe's output bar
    # same launches and constants as the Python model: bit-identical salience (5 s)
    wav = torch.from_numpy(synthetic.synthetic_audio(5.0, seed=31)).float().to(DEV)
    sal_py, Tp = py.salience(py.mel_spectrogram(wav))
    sal, F = nat.salience(wav)
    torch.cuda.synchronize()
    nat.check()
    py.check_error()
    assert sal.shape == (1, 360, Tp) and F == 1 + wav.numel() // 160
    assert torch.equal(sal[0], sal_py)
    # natively derived window / DFT / mel constants (the window differs from torch's Sleef cosf in a few last
    # bits): the salience within test_gpu_rmvpe's bar against the reference (3e-5 RMS)
    nat2 = NativeRMVPE(sd, DEV)
    sal2, _ = nat2.salience(wav)
    assert rms(sal2, sal.cpu().numpy()) < 3e-5
    # B sequences = B single calls
    wb = torch.stack([wav, wav.flip(0)])
    both, _ = nat.salience(wb)
    assert torch.equal(both[0], sal[0]) and torch.equal(both[1], nat.salience(wav.flip(0))[0][0])


def test_c_host_runs_the_synthesizer_through_the_header_alone(tmp_path):
    """examples/c_host/synth_demo (gcc, no Python / torch in the process) loads the .pth tensors from a
    safetensors export and runs rvc_synth_infer: bit-identical to NativeSynth on the same inputs and seed."""
    import os
    import subprocess
    from rvc_amd.native import export_synth_safetensors
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "c_host", "synth_demo")
    assert os.path.exists(exe), "build it: make -C examples/c_host"
    ck = synthetic.make_synth_ckpt(40000, "v2", seed=21)
    export_synth_safetensors(ck, str(tmp_path / "model.safetensors"))
    T, E, sid, seed = 120, 768, 3, 17
    phone, pitch, pitchf = inputs(T, seed=4)
    with open(tmp_path / "inputs.bin", "wb") as f:
        f.write(np.array([T, E, sid, seed], np.int64).tobytes())
        f.write(phone[0].cpu().numpy().astype(np.float32).tobytes())
        f.write(pitch[0].cpu().numpy().astype(np.int64).tobytes())
        f.write(pitchf[0].cpu().numpy().astype(np.float32).tobytes())
    r = subprocess.run([exe, str(tmp_path / "model.safetensors"), str(tmp_path / "inputs.bin"), str(tmp_path / "out.f32")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(tmp_path / "out.f32", dtype=np.float32)
    ref = NativeSynth(ck, DEV).infer(phone, torch.tensor([T]), pitch, pitchf, sid, seed=seed)[0]
    assert got.shape == (T * 400,)
    assert np.array_equal(got, ref.reshape(-1).cpu().numpy()), r.stdout


@pytest.mark.parametrize("capacity,seconds", [("tiny", 6.0), ("full", 2.5)])
def test_native_crepe_bit_identical_to_python(capacity, seconds):
    from rvc_amd.crepe import CrepeAMD
    from rvc_amd.native import NativeCrepe
    sd = synthetic.crepe_state_dict(31, capacity)
    py = CrepeAMD(sd, capacity, DEV)
    nat = NativeCrepe(sd, DEV, log_trans=py.log_trans.cpu(), bn=py.bns)  # the Python model's own constants
    wav = torch.from_numpy(synthetic.synthetic_audio(seconds, seed=41)).float().to(DEV)
    T = 1 + wav.numel() // 160  # 6 s: two 512-frame Viterbi batches
    dither = np.random.default_rng(3).triangular(-20.0, 0.0, 20.0, size=T)
    py.dither_fn = lambda n: dither
    trace = {}
    c_py, f_py = py.f0_device(wav, 2.0, trace=trace)
    c_n, f_n, probs = nat.f0_device(wav, 2.0, dither=dither, want_probs=True)
    torch.cuda.synchronize()
    assert np.array_equal(probs.t().cpu().numpy(), trace["probs"])
    assert torch.equal(c_n, c_py) and torch.equal(f_n, f_py)
    # natively derived BatchNorm fold (IEEE sqrt; torch's CPU sqrt is off by an ulp on a few channels) and
    # transition matrix: the same probabilities to f32 rounding, the same coarse track
    c2, f2, p2 = NativeCrepe(sd, DEV).f0_device(wav, 2.0, dither=dither, want_probs=True)
    assert float((p2 - probs).abs().max()) < 1e-5
    assert float((c2 == c_py).float().mean()) > 0.99
    # device dither (NULL): finite, in the quantiser's range
    c3, f3, _ = nat.f0_device(wav, 0.0, seed=5)
    assert int(c3.min()) >= 1 and int(c3.max()) <= 255 and torch.isfinite(f3).all()


@pytest.mark.parametrize("sr,version,protect,pitch", [(48000, "v2", 0.33, 0.0), (32000, "v1", 0.5, 3.0)])
def test_native_vc_convert_equals_pipeline_device(sr, version, protect, pitch):
    """rvc_vc_convert (one segment through the C ABI) vs VC.pipeline_device on the same models, constants and
    seed: bit-identical waveform."""
    from rvc_amd import melbasis
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.native import NativeVC
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD, fold_weight_norm
    hub_ck = synthetic.make_contentvec_ckpt(51)
    rm_sd = synthetic.rmvpe_state_dict(52)
    cpt = synthetic.make_synth_ckpt(sr, version, seed=53)
    hub, net_g = ContentVecAMD(hub_ck, DEV), SynthesizerAMD(cpt, DEV)
    vc = VC(sr, Config(DEV), rmvpe=RMVPEAMD(rm_sd, DEV))
    hw = dict(hub_ck["model"])
    p = "encoder.pos_conv.0.weight"
    hw[p] = torch._weight_norm(hw.pop(p + "_v").float(), hw.pop(p + "_g").float(), 2)
    nat = NativeVC(hub_ck, rm_sd, cpt, DEV, synth_weights=fold_weight_norm(cpt["weight"]), hub_weights=hw,
                   window=torch.hann_window(1024), mel_basis=melbasis.mel_filterbank(16000, 1024, 128, 30, 8000))
    audio = torch.from_numpy(synthetic.synthetic_audio(4.3, seed=54)).float().to(DEV)
    ref = vc.pipeline_device(hub, net_g, 0, audio, pitch, version, protect)
    got = nat.convert(audio, 0, pitch, protect, version, seed=0)
    torch.cuda.synchronize()
    vc.check_errors()
    assert got.shape == ref.shape
    assert torch.equal(got, ref), rms(got, ref)


def test_c_host_runs_a_whole_segment(tmp_path):
    """examples/c_host/vc_demo: ContentVec, RMVPE and the voice model from safetensors exports, one
    rvc_vc_convert call, from plain C; bit-identical to NativeVC on the same clip and seed."""
    import os
    import subprocess
    from rvc_amd.native import NativeVC, export_safetensors, export_synth_safetensors
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "c_host", "vc_demo")
    assert os.path.exists(exe), "build it: make -C examples/c_host"
    hub_ck = synthetic.make_contentvec_ckpt(61)
    rm_sd = synthetic.rmvpe_state_dict(62)
    cpt = synthetic.make_synth_ckpt(40000, "v2", seed=63)
    export_safetensors(hub_ck["model"], str(tmp_path / "hub.safetensors"), rvc_contentvec_cfg=[768, 12, 16, 0])
    export_safetensors(rm_sd, str(tmp_path / "rmvpe.safetensors"))
    export_synth_safetensors(cpt, str(tmp_path / "model.safetensors"))
    audio = synthetic.synthetic_audio(3.7, seed=64).astype(np.float32)
    audio.tofile(tmp_path / "audio.f32")
    r = subprocess.run([exe, str(tmp_path / "hub.safetensors"), str(tmp_path / "rmvpe.safetensors"),
                        str(tmp_path / "model.safetensors"), str(tmp_path / "audio.f32"), str(tmp_path / "out.f32"),
                        "2", "0.33", "7"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(tmp_path / "out.f32", dtype=np.float32)
    ref = NativeVC(hub_ck, rm_sd, cpt, DEV).convert(torch.from_numpy(audio).to(DEV), 0, 2.0, 0.33, "v2", seed=7)
    assert got.shape == tuple(ref.shape) and np.array_equal(got, ref.cpu().numpy()), r.stdout


def test_native_vc_convert_with_index_equals_pipeline_device():
    """BASELINE configs[2]'s retrieval (IVF-Flat, index_rate 0.75) inside rvc_vc_convert: bit-identical to
    VC.pipeline_device with the same index."""
    from rvc_amd import melbasis
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.faiss_index import IVFFlatIndex
    from rvc_amd.native import NativeVC
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.retrieval import IVFFlatDevice
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD, fold_weight_norm
    hub_ck, rm_sd, cpt = synthetic.make_contentvec_ckpt(71), synthetic.rmvpe_state_dict(72), \
        synthetic.make_synth_ckpt(48000, "v2", seed=73)
    hub, net_g = ContentVecAMD(hub_ck, DEV), SynthesizerAMD(cpt, DEV)
    vc = VC(48000, Config(DEV), rmvpe=RMVPEAMD(rm_sd, DEV))
    feats = hub.features_cf(torch.from_numpy(synthetic.synthetic_audio(8.0, seed=74)).to(DEV)).t().cpu().numpy()
    rng = np.random.default_rng(2)
    idx = IVFFlatIndex.build(feats[rng.choice(len(feats), 24, replace=False)], feats, nprobe=3)
    hw = dict(hub_ck["model"])
    p = "encoder.pos_conv.0.weight"
    hw[p] = torch._weight_norm(hw.pop(p + "_v").float(), hw.pop(p + "_g").float(), 2)
    nat = NativeVC(hub_ck, rm_sd, cpt, DEV, synth_weights=fold_weight_norm(cpt["weight"]), hub_weights=hw,
                   window=torch.hann_window(1024), mel_basis=melbasis.mel_filterbank(16000, 1024, 128, 30, 8000))
    nat.load_index(idx)
    audio = torch.from_numpy(synthetic.synthetic_audio(5.1, seed=75)).float().to(DEV)
    ref = vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33, IVFFlatDevice(idx, DEV), 0.66)
    got = nat.convert(audio, 0, 0.0, 0.33, "v2", seed=0, index_rate=0.66)  # not a float value: f64 end to end
    plain = nat.convert(audio, 0, 0.0, 0.33, "v2", seed=0)
    torch.cuda.synchronize()
    assert torch.equal(got, ref), rms(got, ref)
    assert not torch.equal(got, plain)


def test_load_index_validates_and_replaces():
    """rvc_load_index rejects a malformed index on the host (a load error, not a device read out of bounds
    later) and frees the previous index's device arrays when it replaces one: device memory stays flat
    over repeated reloads of a ~60 MB index."""
    import ctypes
    from rvc_amd import _lib
    from rvc_amd.native import _Ctx
    lib = _lib.load()
    ctx = _Ctx(DEV)
    rng = np.random.default_rng(0)
    d, nlist, n = 768, 64, 20000
    cent = rng.standard_normal((nlist, d)).astype(np.float32)
    codes = rng.standard_normal((n, d)).astype(np.float32)
    off = np.linspace(0, n, nlist + 1).astype(np.int64)
    ids = np.arange(n, dtype=np.int64)

    def load(cent=cent, off=off, codes=codes, ids=ids, big=codes, d=d, nlist=nlist, ntotal=n, nprobe=1):
        x = _lib.IvfIndex()
        x.d, x.nlist, x.ntotal, x.nprobe = d, nlist, ntotal, nprobe
        keep = [np.ascontiguousarray(a) for a in (cent, off, codes, ids, big)]
        x.centroids, x.list_off, x.codes, x.ids, x.big = (ctypes.c_void_p(a.ctypes.data) for a in keep)
        return lib.rvc_load_index(ctx.ctx, ctypes.byref(x))

    bad_off = off.copy()
    bad_off[5] = bad_off[7]  # decreasing at list 5 -> 6
    bad_ids = ids.copy()
    bad_ids[123] = n
    for kw in (dict(off=bad_off), dict(ids=bad_ids), dict(d=767), dict(ntotal=0), dict(d=2048)):
        assert load(**kw) != 0, kw
        assert lib.rvc_last_error()
    assert load() == 0
    torch.cuda.synchronize()
    base = lib.rvc_device_bytes_in_use()
    for _ in range(6):
        assert load() == 0
    torch.cuda.synchronize()
    grown = lib.rvc_device_bytes_in_use() - base
    assert grown < 16 << 20, grown  # one index is ~124 MB (codes + big): a leak would grow by 6x that


def _native_and_python(sr=48000, version="v2", seed=81, crepe_cap=None):
    from rvc_amd import melbasis
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.native import NativeVC
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD, fold_weight_norm
    hub_ck, rm_sd, cpt = synthetic.make_contentvec_ckpt(seed), synthetic.rmvpe_state_dict(seed + 1), \
        synthetic.make_synth_ckpt(sr, version, seed=seed + 2)
    hub, net_g = ContentVecAMD(hub_ck, DEV), SynthesizerAMD(cpt, DEV)
    crepe = None
    if crepe_cap:
        from rvc_amd.crepe import CrepeAMD
        crepe = {crepe_cap: CrepeAMD(synthetic.crepe_state_dict(seed + 3, crepe_cap), crepe_cap, DEV)}
    vc = VC(sr, Config(DEV), rmvpe=RMVPEAMD(rm_sd, DEV), crepe=crepe)
    hw = dict(hub_ck["model"])
    p = "encoder.pos_conv.0.weight"
    hw[p] = torch._weight_norm(hw.pop(p + "_v").float(), hw.pop(p + "_g").float(), 2)
    nat = NativeVC(hub_ck, rm_sd, cpt, DEV, synth_weights=fold_weight_norm(cpt["weight"]), hub_weights=hw,
                   window=torch.hann_window(1024), mel_basis=melbasis.mel_filterbank(16000, 1024, 128, 30, 8000))
    if crepe_cap:
        c = crepe[crepe_cap]
        nat.load_crepe(synthetic.crepe_state_dict(seed + 3, crepe_cap), log_trans=c.log_trans.cpu(), bn=c.bns)
    return vc, hub, net_g, nat


def test_native_vc_convert_long_input_equals_pipeline_device():
    """rvc_vc_convert_ex on a 45 s input: the quiet-point segmentation on the device, f0 over the whole input,
    two segments with their own noise seeds, stitched -- bit-identical to VC.pipeline_device."""
    vc, hub, net_g, nat = _native_and_python()
    audio = torch.from_numpy(synthetic.synthetic_audio(45.0, seed=86)).float().to(DEV)
    ref = vc.pipeline_device(hub, net_g, 0, audio, 1.0, "v2", 0.33)
    got = nat.convert(audio, 0, 1.0, 0.33, "v2", seed=0)
    torch.cuda.synchronize()
    vc.check_errors()
    assert got.shape == ref.shape and torch.equal(got, ref), rms(got, ref)


@pytest.mark.parametrize("f0_method", ["rmvpe", "pm", "crepe"])
def test_native_vc_convert_options_equal_pipeline_device(f0_method):
    """rvc_vc_convert_ex with get_f0's autotune and f0-file override and the volume envelope (convert.py:311-318,
    449), per f0 method: bit-identical to VC.pipeline_device with the same options."""
    vc, hub, net_g, nat = _native_and_python(40000, "v2", 91, crepe_cap="tiny" if f0_method == "crepe" else None)
    audio = torch.from_numpy(synthetic.synthetic_audio(4.6, seed=92)).float().to(DEV)
    inp_f0 = np.array([[0.0, 210.0], [0.37, 260.5], [1.21, 0.0], [2.9, 320.25]], np.float32)
    kw = dict(f0_autotune=True, f0_autotune_strength=0.7, inp_f0=inp_f0, volume_envelope=0.45)
    dither = None
    method = f0_method
    if f0_method == "crepe":
        method = "crepe-tiny"
        T = 1 + (audio.numel() + 2 * vc.t_pad) // 160
        d = torch.from_numpy(np.random.default_rng(5).triangular(-20.0, 0.0, 20.0, T).astype(np.float32))
        vc.crepe["tiny"].dither_fn = lambda n: d.numpy().astype(np.float64)
        dither = d.to(DEV)
    ref = vc.pipeline_device(hub, net_g, 0, audio, -2.0, "v2", 0.33, f0_method=method, **kw)
    got = nat.convert(audio, 0, -2.0, 0.33, "v2", seed=0, f0_method=f0_method, crepe_dither=dither, **kw)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and torch.equal(got, ref), rms(got, ref)
    plain = nat.convert(audio, 0, -2.0, 0.33, "v2", seed=0, f0_method=f0_method, crepe_dither=dither)
    assert not torch.equal(plain, got)


def test_c_host_runs_a_long_input(tmp_path):
    """examples/c_host/vc_demo on a 45 s input (two segments at a device-found quiet point) from safetensors exports
    of the checkpoints with the host's folds (weight norm, pos_conv) and RMVPE's window / mel basis, as the Python
    models make them: bit-identical to VC.pipeline_device."""
    import os
    import subprocess
    from rvc_amd import melbasis
    from rvc_amd.native import export_safetensors, export_synth_safetensors
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD, fold_weight_norm
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "c_host", "vc_demo")
    hub_ck, rm_sd, cpt = synthetic.make_contentvec_ckpt(95), synthetic.rmvpe_state_dict(96), \
        synthetic.make_synth_ckpt(48000, "v2", seed=97)
    hw = dict(hub_ck["model"])
    p = "encoder.pos_conv.0.weight"
    hw[p] = torch._weight_norm(hw.pop(p + "_v").float(), hw.pop(p + "_g").float(), 2)
    export_safetensors(hw, str(tmp_path / "hub.safetensors"), rvc_contentvec_cfg=[768, 12, 16, 0])
    rw = dict(rm_sd, window=torch.hann_window(1024),
              mel_basis=torch.from_numpy(melbasis.mel_filterbank(16000, 1024, 128, 30, 8000)))
    export_safetensors(rw, str(tmp_path / "rmvpe.safetensors"))
    export_synth_safetensors(dict(cpt, weight=fold_weight_norm(cpt["weight"])), str(tmp_path / "model.safetensors"))
    audio = synthetic.synthetic_audio(45.0, seed=98).astype(np.float32)
    audio.tofile(tmp_path / "audio.f32")
    r = subprocess.run([exe, str(tmp_path / "hub.safetensors"), str(tmp_path / "rmvpe.safetensors"),
                        str(tmp_path / "model.safetensors"), str(tmp_path / "audio.f32"), str(tmp_path / "out.f32"),
                        "0", "0.33", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(tmp_path / "out.f32", dtype=np.float32)
    vc = VC(48000, Config(DEV), rmvpe=RMVPEAMD(rm_sd, DEV))
    vc.seed = 3
    ref = vc.pipeline_device(ContentVecAMD(hub_ck, DEV), SynthesizerAMD(cpt, DEV), 0,
                             torch.from_numpy(audio).to(DEV), 0.0, "v2", 0.33).cpu().numpy()
    vc.check_errors()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert np.array_equal(got, ref), (float(np.sqrt(np.mean((got.astype(np.float64) - ref) ** 2))), r.stdout)
