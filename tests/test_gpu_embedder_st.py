"""The transformers ``.safetensors`` embedder: ``HubertModelWithFinalProj.from_pretrained``
(main/library/utils.py:157-165) as VC.voice_conversion uses it (convert.py:342-345), on the device.

The model directory (config.json + model.safetensors in transformers' parameter names, synthetic.make_hf_hubert)
is written at test time; the expected outputs are the reference's own (tests/golden/contentvec_hf.npz and
pipeline_*_st.npz: make_golden.py safetensors ran the reference's load_embedders_model + VC.pipeline with
transformers 5.15 on these weights)."""
import json

import numpy as np
import pytest
import torch

from rvc_amd import synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def write_dir(tmp_path, seed):
    from safetensors.torch import save_file
    cfg, sd = synthetic.make_hf_hubert(seed)
    d = tmp_path / f"hf_{seed}"
    d.mkdir()
    (d / "config.json").write_text(json.dumps(cfg))
    save_file({k: v.contiguous() for k, v in sd.items()}, str(d / "model.safetensors"))
    return str(d)


def rms(a, b):
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    return float(np.sqrt(np.mean((a - np.asarray(b, np.float64)) ** 2)))


def test_from_transformers_features_match_reference(golden, tmp_path):
    from rvc_amd.contentvec import ContentVecAMD
    g = golden("contentvec_hf")
    m = ContentVecAMD.from_transformers(write_dir(tmp_path, int(g["seed"])), DEV)
    assert m.embed_suffix == ".safetensors"
    src = torch.from_numpy(g["audio"]).view(1, -1).to(DEV)
    last = m(src)["last_hidden_state"]  # the call convert.py:343 makes
    assert last.shape == g["last_hidden_state"].shape
    assert rms(last, g["last_hidden_state"]) < 1e-4
    assert rms(m.final_proj(last), g["feats_v1"]) < 1e-4  # convert.py:344 (v1: final_proj of the LAST layer)
    v1 = m.embed_cf(src.reshape(-1), "v1")
    assert rms(v1.t().unsqueeze(0), g["feats_v1"]) < 1e-4


@pytest.mark.parametrize("name", ["pipeline_48k_v2_st", "pipeline_32k_v1_st"])
def test_pipeline_safetensors_matches_reference_golden(golden, name, tmp_path):
    """VC.pipeline(embed_suffix=".safetensors") within the north-star 1e-4 RMS of the reference's output."""
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    g = golden(name)
    sr, version, seed = int(g["sr"]), str(g["version"]), int(g["seed"])
    assert str(g["embed"]) == ".safetensors"
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(sr, version, seed=seed), DEV)
    hub = ContentVecAMD.from_transformers(write_dir(tmp_path, seed + 1), DEV)
    vc = VC(sr, Config(DEV), rmvpe=RMVPEAMD(synthetic.rmvpe_state_dict(seed + 2), DEV))

    def noise(seg, kind, shape):
        a = torch.from_numpy(g[f"{'z' if kind == 'z' else 'sine'}_noise_{seg}"]).to(DEV)
        assert tuple(a.shape) == tuple(shape)
        return a

    vc.noise_fn = noise
    out = vc.pipeline(model=hub, net_g=net_g, sid=0, audio=g["audio"].copy(), pitch=float(g["pitch"]),
                      f0_method="rmvpe", file_index="", index_rate=0.0, pitch_guidance=1, filter_radius=3,
                      volume_envelope=1.0, version=version, protect=float(g["protect"]), hop_length=64,
                      f0_autotune=False, f0_autotune_strength=1.0, suffix=".pth", embed_suffix=".safetensors")
    vc.check_errors()
    assert out.shape == g["out"].shape
    err = rms(out, g["out"])
    assert err < 1e-4, err
    # the same weights through the .pt semantics differ for v1 (layer 9 vs the last layer feeds final_proj)
    if version == "v1":
        out_pt = vc.pipeline(model=hub, net_g=net_g, sid=0, audio=g["audio"].copy(), pitch=float(g["pitch"]),
                             f0_method="rmvpe", file_index="", index_rate=0.0, pitch_guidance=1, filter_radius=3,
                             volume_envelope=1.0, version=version, protect=float(g["protect"]), hop_length=64,
                             f0_autotune=False, f0_autotune_strength=1.0, suffix=".pth", embed_suffix=".pt")
        assert rms(out_pt, g["out"]) > 1e-3


def test_convert_audio_transformers_mode_v1(golden, tmp_path, monkeypatch):
    """VoiceConverterAMD.convert_audio(embedders_mode="transformers") on a transformers-loaded v1 model: the
    pipeline runs with the ".safetensors" suffix load_embedders_model returns (utils.py:155-165), i.e. the last
    layer + final_proj (convert.py:342-345), and matches the reference's golden; a mode that disagrees with the
    loaded model is refused (logged, None), not run with the wrong layer."""
    from rvc_amd import audio_io
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.convert import VoiceConverterAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    g = golden("pipeline_32k_v1_st")
    sr, version, seed = int(g["sr"]), str(g["version"]), int(g["seed"])
    assert np.abs(g["audio"]).max() <= 0.95  # convert_audio's peak limit leaves it as the golden pipeline saw it
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(sr, version, seed=seed), DEV)
    hub = ContentVecAMD.from_transformers(write_dir(tmp_path, seed + 1), DEV)
    vc = VC(sr, Config(DEV), rmvpe=RMVPEAMD(synthetic.rmvpe_state_dict(seed + 2), DEV))
    vc.noise_fn = lambda seg, kind, shape: torch.from_numpy(
        g[f"{'z' if kind == 'z' else 'sine'}_noise_{seg}"]).to(DEV)
    monkeypatch.setattr(audio_io, "load_audio", lambda *a, **k: g["audio"].copy())
    cvt = VoiceConverterAMD(vc, net_g, hub, sr, version=version)
    kw = dict(pitch=float(g["pitch"]), f0_method="rmvpe", index_rate=0.0, volume_envelope=1.0,
              protect=float(g["protect"]))
    out = cvt.convert_audio("in.wav", str(tmp_path / "out.wav"), embedders_mode="transformers", **kw)
    assert out is not None, "convert_audio logged an error"
    assert rms(out, g["out"]) < 1e-4
    assert vc.embed_suffix is None  # the call's suffix does not stay on the VC
    assert cvt.convert_audio("in.wav", str(tmp_path / "out2.wav"), embedders_mode="fairseq", **kw) is None
