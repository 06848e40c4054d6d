"""ContentVec extract_features on the HIP path vs the reference's own outputs (golden vectors)."""
import numpy as np
import pytest
import torch

from rvc_amd import synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rms(a, b):
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.sqrt(np.mean((a - b) ** 2)))


@pytest.fixture(scope="module")
def model(golden):
    from rvc_amd.contentvec import ContentVecAMD
    g = golden("contentvec")
    return ContentVecAMD(synthetic.make_contentvec_ckpt(int(g["seed"])), DEV), g


def test_contentvec_v2_layer12(model):
    m, g = model
    src = torch.from_numpy(g["audio"]).view(1, -1).to(DEV)
    x, pm = m.extract_features(source=src, padding_mask=torch.zeros_like(src, dtype=torch.bool), output_layer=12)
    torch.cuda.synchronize()
    assert rms(x, g["feats_v2"]) < 1e-4


def test_contentvec_v1_layer9_final_proj(model):
    m, g = model
    src = torch.from_numpy(g["audio"]).view(1, -1).to(DEV)
    x, _ = m.extract_features(source=src, padding_mask=None, output_layer=9)
    y = m.final_proj(x)
    torch.cuda.synchronize()
    assert rms(y, g["feats_v1"]) < 1e-4


def test_contentvec_long_vs_oracle(model):
    """6.3 s input (T_f = 315, odd -> the reference pads one masked key) vs the CPU oracle."""
    from oracle import contentvec as ocv
    m, g = model
    wav = synthetic.synthetic_audio(6.3, seed=77)
    W = ocv.load_weights(synthetic.make_contentvec_ckpt(int(g["seed"])))
    with torch.no_grad():
        ref = ocv.extract_features(W, torch.from_numpy(wav).view(1, -1), 12)
    x, _ = m.extract_features(torch.from_numpy(wav).view(1, -1).to(DEV), output_layer=12)
    assert x.shape[1] == ocv.frames(len(wav))
    assert rms(x, ref.numpy()) < 1e-4
