"""RMVPE on the HIP path vs the reference's own outputs (golden vectors)."""
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
    from rvc_amd.rmvpe import RMVPEAMD
    g = golden("rmvpe")
    return RMVPEAMD(synthetic.rmvpe_state_dict(int(g["seed"])), DEV), g


def test_mel(model):
    m, g = model
    mel = m.mel_spectrogram(torch.from_numpy(g["audio"]).float().to(DEV))
    assert rms(mel.unsqueeze(0), g["mel"]) < 1e-4


def test_salience(model):
    m, g = model
    mel = torch.from_numpy(g["mel"][0]).to(DEV)
    sal, Tp = m.salience(mel)
    F = mel.shape[-1]
    got = sal[:, :F].t().unsqueeze(0)
    torch.cuda.synchronize()
    m.check_error()
    # f32-level rounding through ~40 conv/BN layers + the BiGRU; the f0 test below is the output bar
    assert rms(got, g["hidden"]) < 3e-5


def test_f0_end_to_end(model):
    m, g = model
    f0 = m.infer_from_audio(g["audio"], thred=0.03)
    assert f0.shape == g["f0"].shape
    assert np.max(np.abs(f0 - g["f0"])) < 1e-2


def test_decode_known_answer(model):
    """Peaked-salience KAT from the reference decode: f64 arithmetic, numpy reduction order."""
    from rvc_amd import ops
    m, g = model
    sal = torch.from_numpy(np.ascontiguousarray(g["kat_salience"].T)).to(DEV)
    F = sal.shape[1]
    f0 = torch.empty(F, dtype=torch.float64, device=DEV)
    coarse = torch.empty(F, dtype=torch.int64, device=DEV)
    pf = torch.empty(F, device=DEV)
    ops.rmvpe_decode(sal, F, F, 0.03, 1.0, f0, coarse, pf)
    np.testing.assert_allclose(f0.cpu().numpy(), g["kat_f0"], rtol=0, atol=1e-9)


def test_coarse_matches_oracle_quantiser(model):
    """Device mel quantiser vs convert.py:311-323 on an f0 sweep (as salience peaks) with pitch shift."""
    from oracle import pipeline as opl
    from rvc_amd import ops
    m, _ = model
    F = 360
    sal = torch.zeros(360, F)
    for t in range(F):
        sal[t, t] = 0.9
    sal = sal.to(DEV).contiguous()
    f0 = torch.empty(F, dtype=torch.float64, device=DEV)
    coarse = torch.empty(F, dtype=torch.int64, device=DEV)
    pf = torch.empty(F, device=DEV)
    for shift in (0, 3, -12):
        ops.rmvpe_decode(sal, F, F, 0.03, 2 ** (shift / 12), f0, coarse, pf)
        base = 10 * 2 ** ((20 * np.arange(360) + 1997.3794084376191) / 1200)
        want_c, want_f = opl.coarse_f0(base.copy(), shift, opl.Consts(48000))
        np.testing.assert_allclose(f0.cpu().numpy(), want_f, rtol=1e-12)
        assert np.array_equal(coarse.cpu().numpy(), want_c)


def test_bigru_timeout_is_reported_and_cleared(model):
    """A BiGRU hand-off that exceeds its spin limit flags err; check_error raises once, then the flag
    is clear and a normal run passes (the kernel drains instead of hanging)."""
    from rvc_amd import _lib
    m, g = model
    lib = _lib.load()
    audio = torch.from_numpy(g["audio"]).float().to(DEV)
    prev = lib.rvc_bigru_set_spin_limit(1)
    try:
        m.f0_device(audio)
        torch.cuda.synchronize()
    finally:
        lib.rvc_bigru_set_spin_limit(prev)
    assert lib.rvc_bigru_set_spin_limit(0) == prev
    with pytest.raises(RuntimeError, match="bigru"):
        m.check_error()
    m.check_error()  # cleared
    coarse, pitchf, f0 = m.f0_device(audio, want_f0=True)
    torch.cuda.synchronize()
    m.check_error()
    assert np.max(np.abs(f0.cpu().numpy() - g["f0"])) < 1e-2
