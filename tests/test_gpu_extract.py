"""Training-feature extraction (extract.py mirror) and the convert_audio front end on the device
models: f0 / features against the CPU oracle, coarse against the reference's quantiser, and
convert_audio(split_audio=True) against cut -> pipeline per chunk -> restore done by hand."""
import os

import numpy as np
import pytest
import torch

from rvc_amd import audio_io, edges, extract, synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEED = 31


@pytest.fixture(scope="module")
def models():
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.rmvpe import RMVPEAMD
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(SEED + 1), DEV)
    rm = RMVPEAMD(synthetic.rmvpe_state_dict(SEED + 2), DEV)
    return hub, rm


def _exp_dir(root, secs):
    for d in ("sliced_audios", "sliced_audios_16k"):
        os.makedirs(os.path.join(root, d), exist_ok=True)
    names = []
    for i, s in enumerate(secs):
        n = f"0_{i}.wav"
        x = synthetic.synthetic_audio(s, seed=500 + i)
        audio_io.write_wav(os.path.join(root, "sliced_audios_16k", n), x, 16000)
        audio_io.write_wav(os.path.join(root, "sliced_audios", n), x, 48000)
        names.append(n)
    return names


@pytest.mark.parametrize("version", ["v2", "v1"])
def test_extract_matches_oracle(tmp_path, models, version):
    from oracle import contentvec as ocv
    from oracle import rmvpe as orm
    from rvc_amd import melbasis
    hub, rm = models
    root = str(tmp_path)
    names = _exp_dir(root, [1.3, 2.0, 0.9])
    fi = extract.FeatureInputAMD(device=DEV, rmvpe=rm)
    extract.run_extract(root, version, "rmvpe", hub, fi, DEV, write_config=False)
    Wc = ocv.load_weights(synthetic.make_contentvec_ckpt(SEED + 1))
    Wr = orm.load_weights(synthetic.rmvpe_state_dict(SEED + 2))
    mel = torch.from_numpy(melbasis.mel_filterbank())
    for n in names:
        x = audio_io.load_audio(os.path.join(root, "sliced_audios_16k", n))
        f0 = np.load(os.path.join(root, "f0_voiced", n + ".npy"))
        with torch.no_grad():
            ref_f0 = orm.infer_from_audio(Wr, mel, x.astype(np.float64), 0.03)
        assert f0.dtype == np.float64 and f0.shape == ref_f0.shape
        assert int(((f0 > 0) != (ref_f0 > 0)).sum()) <= 1  # a voicing decision within f32 rounding may flip
        both = (f0 > 0) & (ref_f0 > 0)
        assert np.abs(np.log2(f0[both] / ref_f0[both])).max() < 1e-3
        np.testing.assert_array_equal(np.load(os.path.join(root, "f0", n + ".npy")), fi.coarse_f0(f0))
        feats = np.load(os.path.join(root, f"{version}_extracted", n.replace("wav", "npy")))
        with torch.no_grad():
            ref = ocv.extract_features(Wc, torch.from_numpy(x).view(1, -1), 9 if version == "v1" else 12)
            if version == "v1":
                ref = ocv.final_proj(Wc, ref)
        ref = ref[0].numpy()
        assert feats.dtype == np.float32 and feats.shape == ref.shape
        assert float(np.sqrt(np.mean((feats.astype(np.float64) - ref) ** 2))) < 1e-4
    lines = open(os.path.join(root, "filelist.txt")).read().split("\n")
    assert len(lines) == len(names) + 2


def test_extract_crepe_f0(tmp_path, models):
    from rvc_amd.crepe import CrepeAMD
    hub, _ = models
    root = str(tmp_path)
    names = _exp_dir(root, [1.1])
    cr = CrepeAMD(synthetic.crepe_state_dict(1240, "tiny"), "tiny", DEV)
    fi = extract.FeatureInputAMD(device=DEV, crepe={"tiny": cr})
    extract.run_pitch_extraction(root, "crepe-tiny", 160, fi)
    x = audio_io.load_audio(os.path.join(root, "sliced_audios_16k", names[0]))
    f0 = np.load(os.path.join(root, "f0_voiced", names[0] + ".npy"))
    assert f0.dtype == np.float32 and f0.shape == (1 + x.size // 160,)
    np.testing.assert_array_equal(np.load(os.path.join(root, "f0", names[0] + ".npy")), fi.coarse_f0(f0))
    with pytest.raises(NotImplementedError):
        fi.compute_f0(x, "harvest")


def test_convert_audio_split_matches_manual(tmp_path, models):
    from rvc_amd.convert import VoiceConverterAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.synth import SynthesizerAMD
    hub, rm = models
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(48000, "v2", seed=SEED), DEV)
    vc = VC(48000, Config(DEV), rmvpe=rm)
    # a cut after >= 5 s of clip (min_length) and a trailing silence: 2 chunks with a zero gap between
    audio = synthetic.silence_layout_audio([(0.5, 0), (5.5, 1), (0.8, 0), (1.5, 1), (0.6, 0)], seed=9)
    audio = audio * np.float32(0.5 / np.abs(audio).max())
    src = str(tmp_path / "in.wav")
    audio_io.write_wav(src, audio, 16000)
    x = audio_io.load_audio(src)
    cvt = VoiceConverterAMD(vc, net_g, hub, 48000, "v2")
    vc.seed = 5
    out = cvt.convert_audio(src, str(tmp_path / "out.wav"), pitch=0, f0_method="rmvpe", index_rate=0.0,
                            protect=0.33, split_audio=True)
    assert out is not None
    vc.seed = 5
    kw = dict(model=hub, net_g=net_g, sid=0, pitch=0, f0_method="rmvpe", file_index="", index_rate=0.0,
              pitch_guidance=1, filter_radius=3, volume_envelope=1, version="v2", protect=0.33, hop_length=64,
              f0_autotune=False, f0_autotune_strength=1, suffix=".pth", embed_suffix=".pt")
    chunks = edges.cut(x, 16000, -60, 500)
    assert len(chunks) == 2
    ref = edges.restore([(s, e, vc.pipeline(audio=c, **kw)) for c, s, e in chunks], len(x))
    np.testing.assert_array_equal(out, ref)
    y, sr = audio_io.read_wav(str(tmp_path / "out.wav"))
    assert sr == 48000 and y.shape == ref.shape
    assert np.abs(y - np.clip(ref, -1, 1)).max() <= 2.0 / 32767
