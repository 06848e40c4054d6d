"""Spectral-gate denoise (main/tools/noisereduce.py, convert_audio's clean_audio) on the CPU side: the
oracle restatement against the reference's own output (tests/golden/denoise.npz, made by running
noisereduce.reduce_noise in the survey container), and the host-side constants of rvc_amd.denoise."""
import numpy as np
import pytest

from oracle import denoise as od


@pytest.mark.parametrize("case", ["a", "b", "c"])
def test_oracle_matches_reference(golden, case):
    g = golden("denoise")
    sr, prop, cs, pad = g[f"{case}_meta"]
    out = od.reduce_noise(g[f"{case}_y"], sr, prop_decrease=prop, chunk_size=int(cs), padding=int(pad))
    ref = g[f"{case}_out"]
    assert out.dtype == np.float32 and out.shape == ref.shape
    # the reference gates in float64 and rounds once to float32: at most one f32 ulp apart
    assert np.abs(out - ref).max() <= np.spacing(np.float32(np.abs(ref).max()))


@pytest.mark.parametrize("sr", [8000, 16000, 40000, 44100, 48000, 96000])
def test_host_smoothing_filter_matches_oracle(sr):
    from rvc_amd.denoise import smoothing_filter
    a = smoothing_filter(sr, 1024, 256)
    b = od.smoothing_filter(sr, 1024, 256)
    assert a.shape == b.shape and a.shape[0] % 2 == 1 and a.shape[1] % 2 == 1
    np.testing.assert_array_equal(a.numpy(), b)
    assert abs(float(a.sum()) - 1.0) < 1e-6


def test_abi_rejects_bad_args_without_gpu():
    import ctypes
    from rvc_amd import _lib
    lib = _lib.load()
    a = _lib.DenoiseArgs()
    a.chunk_size, a.padding, a.n_fft, a.hop, a.n_movemean = 600000, 30000, 1000, 250, 375  # n_fft not 2^k
    assert lib.rvc_denoise_work_bytes(48000, ctypes.byref(a)) == -1
    a.n_fft, a.hop = 1024, 256
    assert lib.rvc_denoise_work_bytes(48000, ctypes.byref(a)) > 0
    assert lib.rvc_denoise(None, 48000, ctypes.byref(a), None, 0, None, None) == -22
