"""Audio edges against the reference's own outputs (tests/golden/edges.npz, made by
running main/library/utils.py cut/restore, main/inference/preprocess.py Slicer/get_rms and
main/inference/extract.py FeatureInput.coarse_f0): exact chunk boundaries, bitwise RMS frames."""
import numpy as np
import pytest

from rvc_amd import edges, synthetic


@pytest.fixture(scope="module")
def g(golden):
    return golden("edges")


@pytest.mark.parametrize("name", list(synthetic.SLICER_LAYOUTS))
def test_cut_restore_match_reference(g, name):
    audio = synthetic.silence_layout_audio(synthetic.SLICER_LAYOUTS[name], seed=int(g["seed"]))
    np.testing.assert_array_equal(edges.get_rms(audio, 1280, 320).squeeze(0), g[f"{name}_rms"])
    chunks = edges.cut(audio, 16000, db_thresh=-60, min_interval=500)
    np.testing.assert_array_equal(np.array([[s, e] for _, s, e in chunks]), g[f"{name}_bounds"])
    np.testing.assert_array_equal([len(c) for c, _, _ in chunks], g[f"{name}_lens"])
    np.testing.assert_array_equal([float(np.sum(c, dtype=np.float64)) for c, _, _ in chunks], g[f"{name}_sums"])
    conv = [(s, e, np.repeat(c, 3) * 0.5) for c, s, e in chunks]
    rest = edges.restore(conv, total_len=len(audio), dtype=conv[0][2].dtype) if len(chunks) > 1 else conv[0][2]
    assert len(rest) == int(g[f"{name}_restore_len"])
    assert float(np.sum(rest, dtype=np.float64)) == float(g[f"{name}_restore_sum"])
    np.testing.assert_array_equal(np.flatnonzero(rest == 0)[::997][:200], g[f"{name}_restore_nz"])


@pytest.mark.parametrize("name", list(synthetic.SLICER_LAYOUTS))
def test_preprocess_slicer_matches_reference(g, name):
    a40 = synthetic.silence_layout_audio(synthetic.SLICER_LAYOUTS[name], seed=int(g["seed"]), sr=40000)
    sl = edges.Slicer(sr=40000, threshold=-42, min_length=1500, min_interval=400, hop_size=15, max_sil_kept=500)
    ch = sl.slice(a40)
    np.testing.assert_array_equal([len(c) for c in ch], g[f"{name}_pre_lens"])
    np.testing.assert_array_equal([float(np.sum(c, dtype=np.float64)) for c in ch], g[f"{name}_pre_sums"])


def test_get_rms_bitwise(g):
    np.testing.assert_array_equal(edges.get_rms(g["rms_in"], 2048, 512), g["rms_2048_512"])


def test_slicer_arguments_validated():
    with pytest.raises(ValueError):
        edges.Slicer(16000, min_length=100, min_interval=300)
    with pytest.raises(ValueError):
        edges.Slicer(16000, hop_size=20, max_sil_kept=10)


def test_slice2_stereo_and_restore_gaps():
    """Multi-channel input slices on the channel mean; restore fills 16 kHz-domain gaps with zeros."""
    a = synthetic.silence_layout_audio(synthetic.SLICER_LAYOUTS["mixed"], seed=3)
    st = np.stack([a, a * 0.5])
    mono = edges.cut(st.mean(axis=0), 16000, -60, 500)
    multi = edges.cut(st, 16000, -60, 500)
    assert [(s, e) for _, s, e in mono] == [(s, e) for _, s, e in multi]
    assert all(c.shape[0] == 2 for c, _, _ in multi)
    out = edges.restore([(10, 20, np.ones(5, np.float32)), (30, 40, np.ones(3, np.float32))], 50)
    np.testing.assert_array_equal(out, np.r_[np.zeros(10), np.ones(5), np.zeros(10), np.ones(3), np.zeros(10)])
