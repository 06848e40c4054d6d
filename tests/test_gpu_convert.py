"""VoiceConverterAMD.convert_audio end to end against the REFERENCE's own VoiceConverter.convert_audio
(convert.py:479-523) run on the same seeded models (tests/golden/convert.npz, make_golden.py gen_convert):
the 0.95 peak limit, cut() into two chunks, one VC.pipeline per chunk, restore(), and clean_audio's spectral
gate, in the reference's order, with every noise draw of the reference replayed."""
import numpy as np
import pytest
import torch

from rvc_amd import audio_io, synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def converter(golden):
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.convert import VoiceConverterAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    g = golden("convert")
    seed, sr = int(g["seed"]), int(g["sr"])
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(sr, "v2", seed=seed), DEV)
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(seed + 1), DEV)
    vc = VC(sr, Config(DEV), rmvpe=RMVPEAMD(synthetic.rmvpe_state_dict(seed + 2), DEV))
    return g, VoiceConverterAMD(vc, net_g, hub, sr)


@pytest.mark.parametrize("tag,clean", [("plain", False), ("clean", True)])
def test_convert_audio_matches_reference(converter, tmp_path, monkeypatch, tag, clean):
    g, cvt = converter
    monkeypatch.setattr(audio_io, "load_audio", lambda *a, **k: g["audio"].copy())
    used = {"z": 0, "sine": 0}

    def noise(seg, kind, shape):  # the reference's draws, in order, one pipeline call per chunk
        c = used[kind]
        used[kind] += 1
        return torch.from_numpy(g[f"{kind}_noise_{c}"]).reshape(shape).to(DEV)

    cvt.vc.noise_fn = noise
    try:
        out = cvt.convert_audio("in.wav", str(tmp_path / "out.wav"), "", "contentvec_base", 1, "rmvpe", 0.0, 1, 0.33,
                                64, False, 1, 3, clean, 0.5, "wav", split_audio=True)
    finally:
        cvt.vc.noise_fn = None
    assert out is not None, "convert_audio logged an error"
    assert used == {"z": int(g["nchunks"]), "sine": int(g["nchunks"])}
    ref = g[f"{tag}_out"]
    assert out.shape == ref.shape and out.dtype == ref.dtype
    err = float(np.sqrt(np.mean((out.astype(np.float64) - ref) ** 2)))
    assert err <= 1e-4, err
