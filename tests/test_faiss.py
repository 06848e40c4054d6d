"""FAISS IVF-Flat .index reader/writer and the search oracle (CPU).  faiss itself is absent here
(faiss-cpu>=1.7.3, requirements.txt:17): the binary layout is restated from faiss's published
index_write.cpp and is parity-unpinned; the search semantics are checked against brute force."""
import io
import struct

import numpy as np
import pytest

from oracle import ivf
from rvc_amd.faiss_index import IVFFlatIndex, fourcc, read_index


def make_index(n=3000, d=32, nlist=40, nprobe=1, seed=0, empty_lists=False):
    rng = np.random.default_rng(seed)
    xb = rng.standard_normal((n, d)).astype(np.float32)
    cent = xb[rng.choice(n, nlist, replace=False)].copy()
    if empty_lists:
        cent[: nlist // 2 + 2] += 50.0  # far away: those lists receive no vectors
    return IVFFlatIndex.build(cent, xb, nprobe=nprobe), xb


@pytest.mark.parametrize("empty_lists", [False, True], ids=["full", "sparse"])
def test_write_read_round_trip(tmp_path, empty_lists):
    idx, xb = make_index(empty_lists=empty_lists)
    p = tmp_path / "added_IVF40_Flat_nprobe_1_test_v2.index"
    idx.write(str(p))
    raw = p.read_bytes()
    assert struct.unpack("<I", raw[:4])[0] == fourcc("IwFl")
    layout = raw.find(b"sprs") if empty_lists else raw.find(b"full")
    assert layout > 0
    back = read_index(str(p))
    assert (back.d, back.nlist, back.nprobe, back.ntotal) == (idx.d, idx.nlist, idx.nprobe, idx.ntotal)
    np.testing.assert_array_equal(back.centroids, idx.centroids)
    for a, b, ia, ib in zip(back.codes, idx.codes, back.ids, idx.ids):
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(ia, ib)
    np.testing.assert_array_equal(back.reconstruct_n(0, back.ntotal), xb)  # convert.py:395


def test_reader_rejects_other_indexes():
    with pytest.raises(ValueError):
        IVFFlatIndex.read(struct.pack("<I", fourcc("IxF2")) + b"\0" * 64)
    idx, _ = make_index(n=200, nlist=4)
    buf = io.BytesIO()
    idx.write(buf)
    with pytest.raises(ValueError):
        IVFFlatIndex.read(buf.getvalue()[:-10])  # truncated


def test_search_all_lists_equals_brute_force():
    idx, xb = make_index(n=2000, d=16, nlist=25)
    rng = np.random.default_rng(1)
    q = rng.standard_normal((50, 16)).astype(np.float32)
    D, I = ivf.search(idx, q, k=8, nprobe=idx.nlist)
    d_all = ((q[:, None, :].astype(np.float64) - xb[None].astype(np.float64)) ** 2).sum(-1)
    ref_i = np.argsort(d_all, axis=1, kind="stable")[:, :8]
    np.testing.assert_array_equal(I, ref_i)
    np.testing.assert_allclose(D, np.take_along_axis(d_all, ref_i, 1).astype(np.float32), rtol=1e-6)


def test_search_nprobe1_short_lists_pad_like_faiss():
    # 3 vectors in a 2-list index: a query probing a list of 1 gets (FLT_MAX, -1) padding
    cent = np.array([[0.0, 0.0], [10.0, 10.0]], np.float32)
    xb = np.array([[0.1, 0.0], [9.9, 10.0], [10.2, 10.1]], np.float32)
    idx = IVFFlatIndex.build(cent, xb)
    D, I = ivf.search(idx, np.array([[0.0, 0.1]], np.float32), k=8)
    assert I[0, 0] == 0 and (I[0, 1:] == -1).all()
    assert (D[0, 1:] == np.finfo(np.float32).max).all()


def test_blend_matches_reference_formula():
    rng = np.random.default_rng(2)
    big = rng.standard_normal((100, 8)).astype(np.float32)
    feats = rng.standard_normal((5, 8)).astype(np.float32)
    I = rng.integers(0, 100, (5, 8))
    D = (rng.random((5, 8)) + 0.1).astype(np.float32)
    out = ivf.blend(feats, D, I, big, 0.75)
    w = (1 / D.astype(np.float64)) ** 2
    w /= w.sum(1, keepdims=True)
    ref = 0.75 * (big[I] * w[..., None]).sum(1) + 0.25 * feats
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)


def test_faiss_arithmetic_restatement():
    """oracle/ivf.py's faiss-f32 arithmetic: the AVX2-structured f32 sums equal an explicit loop in that order,
    the BLAS coarse decomposition (nq >= 20) clamps the roundoff of an exact hit at 0, the direct path (nq < 20)
    gives 0 exactly, and both stay within f32 rounding of the exact (f64) distances."""
    rng = np.random.default_rng(5)
    for d in (768, 13):
        x, y = rng.standard_normal(d).astype(np.float32), rng.standard_normal(d).astype(np.float32)
        t = (x - y) * (x - y)
        lanes = [np.float32(0)] * 8
        for j in range(d // 8 * 8):
            lanes[j % 8] = np.float32(lanes[j % 8] + t[j])
        s4 = [np.float32(lanes[4 + i] + lanes[i]) for i in range(4)]
        rest = list(t[d // 8 * 8:]) + [np.float32(0)] * 8
        if d % 8 >= 4:
            s4 = [np.float32(s4[i] + rest[i]) for i in range(4)]
            rest = rest[4:]
        if d % 4:
            s4 = [np.float32(s4[i] + rest[i]) for i in range(4)]
        want = np.float32(np.float32(s4[0] + s4[1]) + np.float32(s4[2] + s4[3]))
        assert ivf.fvec_l2sqr(x[None], y[None])[0] == want
    c = rng.standard_normal((30, 64)).astype(np.float32) * 3
    q = np.concatenate([c[:25], rng.standard_normal((5, 64)).astype(np.float32)])
    blas = ivf.coarse_distances(q, c)                 # 30 queries: the BLAS decomposition
    direct = ivf.coarse_distances(q[:10], c)          # 10 queries: fvec_L2sqr
    exact = ivf.coarse_distances(q, c, "exact")
    assert (blas >= 0).all() and (direct[np.arange(10), np.arange(10)] == 0).all()
    np.testing.assert_allclose(blas, exact, rtol=2e-5, atol=2e-3)
    np.testing.assert_allclose(direct, exact[:10], rtol=1e-5, atol=1e-5)
    idx, _ = make_index(n=800, d=32, nlist=12)
    qq = rng.standard_normal((40, 32)).astype(np.float32)
    Df, If = ivf.search(idx, qq, k=8)
    De, Ie = ivf.search(idx, qq, k=8, arithmetic="exact")
    assert (If == Ie).mean() > 0.99  # near-ties within f32 rounding may order differently
    np.testing.assert_allclose(Df, De, rtol=1e-5, atol=1e-5)
