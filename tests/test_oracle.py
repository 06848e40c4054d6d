"""The oracle (CPU restatement) pinned against golden vectors produced by the reference itself."""
import numpy as np
import pytest
import torch

from oracle import contentvec as ocv
from oracle import pipeline as opl
from oracle import rmvpe as orm
from oracle import synth as osy
from rvc_amd import melbasis, synthetic


def rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


@pytest.mark.parametrize("name", ["synth_48k_v2", "synth_40k_v2", "synth_32k_v1"])
def test_synth_infer_matches_reference(golden, name):
    g = golden(name)
    ck = synthetic.make_synth_ckpt(int(g["sr"]), str(g["version"]), seed=int(g["seed"]))
    W = osy.load_weights(ck["weight"])
    with torch.no_grad():
        o, _, (z, z_p, m_p, logs_p) = osy.infer(
            W, ck["config"], torch.from_numpy(g["phone"]), torch.tensor([int(g["T"])]), torch.from_numpy(g["pitch"]),
            torch.from_numpy(g["pitchf"]), torch.from_numpy(g["sid"]), torch.from_numpy(g["z_noise"]),
            torch.from_numpy(g["sine_noise"]))
    assert rms(m_p, g["m_p"]) < 1e-5
    assert rms(logs_p, g["logs_p"]) < 1e-5
    assert rms(z, g["z"]) < 1e-5
    assert o.shape == g["o"].shape
    assert rms(o, g["o"]) < 1e-5


def test_contentvec_matches_reference(golden):
    g = golden("contentvec")
    W = ocv.load_weights(synthetic.make_contentvec_ckpt(int(g["seed"])))
    src = torch.from_numpy(g["audio"]).view(1, -1)
    with torch.no_grad():
        conv = torch.nn.functional.layer_norm(ocv.feature_extractor(W, src).transpose(1, 2), (512,),
                                              W["layer_norm.weight"], W["layer_norm.bias"], 1e-5)
        conv = torch.nn.functional.linear(conv, W["post_extract_proj.weight"], W["post_extract_proj.bias"])
        v2 = ocv.extract_features(W, src, 12)
        v1 = ocv.final_proj(W, ocv.extract_features(W, src, 9))
    assert rms(conv, g["conv_feats"]) < 1e-5
    assert rms(v2, g["feats_v2"]) < 1e-4
    assert rms(v1, g["feats_v1"]) < 1e-4
    assert ocv.frames(len(g["audio"])) == g["feats_v2"].shape[1]


def test_rmvpe_matches_reference(golden):
    g = golden("rmvpe")
    W = orm.load_weights(synthetic.rmvpe_state_dict(int(g["seed"])))
    mb = torch.from_numpy(melbasis.mel_filterbank())
    with torch.no_grad():
        mel = orm.mel_spectrogram(torch.from_numpy(g["audio"]).float().unsqueeze(0), mb)
        hid = orm.mel2hidden(W, mel)
    assert rms(mel, g["mel"]) < 1e-5
    assert rms(hid, g["hidden"]) < 1e-5
    f0 = orm.decode(hid.squeeze(0).numpy(), 0.03)
    assert np.max(np.abs(f0 - g["f0"])) < 1e-2
    # decode known-answer on a peaked salience: exact f64 arithmetic
    np.testing.assert_allclose(orm.decode(g["kat_salience"], 0.03), g["kat_f0"], rtol=0, atol=1e-12)


def test_own_gru_matches_torch_gru(golden):
    W = orm.load_weights(synthetic.rmvpe_state_dict(31))
    x = torch.randn(1, 40, 384, generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        a = orm.bigru(W, x)
        b = orm.bigru_torch(W, x)
    assert float((a - b).abs().max()) < 1e-5


def test_filtfilt_matches_reference(golden):
    from scipy import signal
    g = golden("filtfilt")
    np.testing.assert_array_equal(opl.BH, g["bh"])
    np.testing.assert_array_equal(opl.AH, g["ah"])
    np.testing.assert_allclose(signal.filtfilt(opl.BH, opl.AH, g["x"]), g["y"], rtol=0, atol=1e-12)


def golden_opts(g):
    """The VC.pipeline options a golden case was generated with (make_golden.gen_pipeline)."""
    opts = {}
    if "f0_autotune_strength" in g:
        opts["autotune_strength"] = float(g["f0_autotune_strength"])
    if "f0_lines" in g:
        opts["inp_f0"] = np.array([[float(v) for v in ln.split(",")] for ln in g["f0_lines"]], dtype=np.float32)
    if "volume_envelope" in g:
        opts["volume_envelope"] = float(g["volume_envelope"])
    return opts


def test_contentvec_safetensors_matches_reference(golden):
    """The .safetensors embedder (transformers HubertModelWithFinalProj, loaded by the reference's own
    load_embedders_model: tests/golden/make_golden.py safetensors): last_hidden_state = every encoder layer,
    v1 = final_proj of it (convert.py:342-345) -- the oracle on the same values under fairseq names."""
    g = golden("contentvec_hf")
    W = ocv.load_weights(synthetic.make_contentvec_ckpt(int(g["seed"])))
    src = torch.from_numpy(g["audio"]).view(1, -1)
    with torch.no_grad():
        last = ocv.extract_features(W, src, ocv.n_layers(W))
        v1 = ocv.final_proj(W, last)
    assert ocv.n_layers(W) == 12
    assert rms(last, g["last_hidden_state"]) < 1e-4
    assert rms(v1, g["feats_v1"]) < 1e-4


def test_hf_names_map_to_fairseq():
    """ContentVecAMD.from_transformers' name map: every transformers parameter lands on the fairseq name holding
    the same values (make_hf_hubert is what transformers loaded without a missing or unexpected key), and an
    unknown parameter raises."""
    from rvc_amd import contentvec
    cfg, sd = synthetic.make_hf_hubert(7)
    fs = contentvec.hf_to_fairseq(sd)
    src = synthetic.contentvec_state_dict(7)
    assert set(fs) == set(src) - {"label_embs_concat"}
    for k, v in fs.items():
        assert torch.equal(v, src[k]), k
    # the older weight_g / weight_v spelling of the pos_conv weight norm, and a "hubert." prefix
    old = {("hubert." + k).replace("parametrizations.weight.original0", "weight_g")
           .replace("parametrizations.weight.original1", "weight_v"): v for k, v in sd.items()}
    assert set(contentvec.hf_to_fairseq(old)) == set(fs)
    with pytest.raises(ValueError):
        contentvec.hf_to_fairseq({**sd, "encoder.layers.0.attention.rel_bias": torch.zeros(1)})
    assert contentvec.hf_config_to_fairseq(cfg)["encoder_embed_dim"] == 768
    with pytest.raises(NotImplementedError):
        contentvec.hf_config_to_fairseq({**cfg, "do_stable_layer_norm": True})


@pytest.mark.parametrize("name", ["pipeline_48k_v2", "pipeline_32k_v1", "pipeline_48k_v2_opts",
                                  "pipeline_48k_v2_st", "pipeline_32k_v1_st"])
def test_pipeline_matches_reference(golden, name):
    g = golden(name)
    sr, version, seed = int(g["sr"]), str(g["version"]), int(g["seed"])
    ck = synthetic.make_synth_ckpt(sr, version, seed=seed)
    Ws = osy.load_weights(ck["weight"])
    Wc = ocv.load_weights(synthetic.make_contentvec_ckpt(seed + 1))
    Wr = orm.load_weights(synthetic.rmvpe_state_dict(seed + 2))
    mb = torch.from_numpy(melbasis.mel_filterbank())

    def noise(seg, kind, shape):
        a = torch.from_numpy(g[f"{'z' if kind == 'z' else 'sine'}_noise_{seg}"])
        assert tuple(a.shape) == tuple(shape)
        return a

    out = opl.pipeline(Wc, Ws, Wr, mb, ck["config"], 0, g["audio"].astype(np.float32), float(g["pitch"]), version,
                       float(g["protect"]), noise, embed_suffix=str(g["embed"]) if "embed" in g else ".pt",
                       **golden_opts(g))
    assert out.shape == g["out"].shape
    assert rms(out, g["out"]) < 1e-5


def test_f0_options_match_reference(golden):
    """Autotune.autotune_f0 on f64 and f32 tracks (convert.py:168-179), get_f0 with autotune + pitch shift +
    f0-file override (convert.py:304-323), change_rms (convert.py:150-152) -- vs the reference's outputs."""
    g = golden("f0_opts")
    np.testing.assert_array_equal(opl.autotune_f0(g["f64"].copy(), 0.75), g["at64"])
    at32 = opl.autotune_f0(g["f32"].copy(), 0.75)
    assert at32.dtype == np.float32
    np.testing.assert_array_equal(at32, g["at32"])
    c = opl.Consts(48000)
    coarse, f0 = opl.coarse_f0(g["track"].copy(), 3, c, 0.6, g["inp_f0"])
    np.testing.assert_array_equal(f0, g["f0"])
    np.testing.assert_array_equal(coarse, g["coarse"])
    out = opl.change_rms(g["rms_src"], 16000, g["rms_tgt"].copy(), 16000, 0.35)
    assert out.dtype == g["rms_out"].dtype
    np.testing.assert_array_equal(out, g["rms_out"])


def test_coarse_quantiser_sweep():
    """VC.get_f0's mel quantiser (convert.py:318-323) on a 0-1500 Hz sweep: unvoiced -> 1, saturates at 255."""
    c = opl.Consts(48000)
    f0 = np.linspace(0, 1500, 3001)
    coarse, f0s = opl.coarse_f0(f0.copy(), 0, c)
    assert coarse[0] == 1 and coarse[-1] == 255
    assert np.all(np.diff(coarse) >= 0)
    assert coarse.dtype == np.int32
    # mute fixture semantics (assets/logs/mute/f0/mute.wav.npy): silence -> coarse 1
    z, _ = opl.coarse_f0(np.zeros(301), 0, c)
    assert np.all(z == 1)


def test_crepe_oracle_matches_reference_golden(golden):
    """VC.get_f0_crepe (convert.py:230-237, CREPE.py) -- network, per-batch viterbi, dither, mean/median."""
    from oracle import crepe as oc
    from rvc_amd import synthetic
    g = golden("crepe")
    sd = synthetic.crepe_state_dict(int(g["seed"]))
    import torch
    frames = oc.preprocess(torch.tensor(np.copy(g["audio"]))[None].float(), 160, 512)
    np.testing.assert_allclose(frames[0][:40].numpy(), g["frames_head"], rtol=0, atol=1e-6)
    tr = {}
    f0 = oc.get_f0_crepe(sd, g["audio"], g["dither"], trace=tr)
    np.testing.assert_allclose(tr["probs"], g["probs"], rtol=0, atol=2e-6)
    assert f0.shape == g["f0"].shape
    np.testing.assert_allclose(f0, g["f0"], rtol=1e-5, atol=1e-3)


def test_rmvpe_f64_matches_reference_f64_and_spread_fixture():
    """The oracle's RMVPE evaluated in float64 (the "exact model" tests/f0check.py measures every f32 evaluation
    against) reproduces the REFERENCE's own f64 evaluation on the headline clip (tests/golden/ref_spread_cfg2.npz,
    make_golden.py spread: its RMVPE model.double() on the same filtered input) at the f64 run's top-2 bins,
    and the fixture's statistics are those the GPU tests read."""
    import f0check
    z = np.load(f0check.GOLDEN)
    ref = f0check.reference_noise()
    audio = synthetic.synthetic_audio(float(z["seconds"]), seed=1000)
    torch.set_num_threads(8)
    s64 = f0check.oracle_salience(synthetic.rmvpe_state_dict(int(z["seed"]) + 2), audio, torch.float64)
    top2, st = z["top2"].astype(np.int64), z["sal_top2"]
    fi = np.arange(s64.shape[0])
    assert np.array_equal(np.argsort(s64, 1)[:, -1], top2[0])  # same f64 argmax on every frame
    # the reference's f64 run builds its Hann window in f64, the oracle upcasts torch's f32 window (RMVPE.py:166)
    assert np.abs(s64[fi, top2[0]] - st[-1, 0]).max() < 1e-6
    assert np.abs(s64[fi, top2[1]] - st[-1, 1]).max() < 1e-6
    # the reference's f32 runs: decision errors of 1e-4 order; a decision different from f64 only where the
    # exact margin is below that noise (one input-ulp run flips frame 326), waveforms within 1e-4 of each other
    # among the runs that take every f64 decision
    assert 1e-5 < ref["decision_noise_max"] < 1e-3 and ref["decision_noise_rms"] < 2e-5
    for name, fl in ref["reference_flips"].items():
        assert name.startswith("f32_") and all(ref["margin64"][fl] < ref["decision_noise_max"]), (name, fl)
    assert ref["wav_spread"] < 1e-4
    assert ref["wav_spread_all"] < 5e-2
