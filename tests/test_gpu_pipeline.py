"""End-to-end VC.pipeline on the HIP path vs the reference's own outputs (golden vectors)."""
import numpy as np
import pytest
import torch

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


@pytest.mark.parametrize("name", ["pipeline_48k_v2", "pipeline_32k_v1"])
def test_pipeline_matches_reference_golden(golden, name):
    g = golden(name)
    sr, version, seed = int(g["sr"]), str(g["version"]), int(g["seed"])
    vc, hub, net_g = build(sr, version, seed)

    def noise(seg, kind, shape):
        a = torch.from_numpy(g[f"{'z' if kind == 'z' else 'sine'}_noise_{seg}"]).to(DEV)
        assert tuple(a.shape) == tuple(shape)
        return a

    vc.noise_fn = noise
    pb = Pbar()
    out = vc.pipeline(model=hub, net_g=net_g, sid=0, audio=g["audio"].copy(), pitch=float(g["pitch"]),
                      f0_method="rmvpe", file_index="", index_rate=0.0, pitch_guidance=1, filter_radius=3,
                      volume_envelope=1, version=version, protect=float(g["protect"]), hop_length=64,
                      f0_autotune=False, f0_autotune_strength=1, suffix=".pth", embed_suffix=".pt", pbar=pb)
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
    ref = opl.pipeline(ocv.load_weights(synthetic.make_contentvec_ckpt(seed + 1)), osy.load_weights(ck["weight"]),
                       orm.load_weights(synthetic.rmvpe_state_dict(seed + 2)),
                       torch.from_numpy(melbasis.mel_filterbank()), ck["config"], 0, audio, 0.0, version, 0.33, noise)
    assert out.shape == ref.shape
    err = float(np.sqrt(np.mean((out.astype(np.float64) - ref) ** 2)))
    assert err < 1e-4, err
