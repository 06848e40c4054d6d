"""TEST INFRASTRUCTURE ONLY (parity oracle; never imported by the product path).

FAISS IVF-Flat search + the reference's retrieval blend, restated in numpy.

``search`` follows faiss's ``IndexIVF::search`` for an ``IndexIVFFlat`` with an ``IndexFlatL2`` quantizer
as the reference builds and calls it (``create_index.py:66-83``: IVF{n},Flat, L2, nprobe 1;
``convert.py:353``: ``index.search(npy, k=8)``).  faiss (``faiss-cpu>=1.7.3``, ``requirements.txt:17``) is
absent here, so this is a restatement of its published algorithm -- "parity unpinned":

* arithmetic "faiss" (the default) -- faiss's own f32 evaluation:
    - coarse step, ``IndexFlatL2::search`` -> ``knn_L2sqr``: for nq >= 20 queries
      (``distance_compute_blas_threshold``) the BLAS decomposition ``exhaustive_L2sqr_blas``:
      dis = ||x||^2 + ||c||^2 - 2 <x, c> in f32, clamped at 0 ("negative values can occur for identical
      vectors due to roundoff"), the best list kept with a strict ``<`` in list order (first index wins a
      tie); below 20 queries ``exhaustive_L2sqr_seq``: dis = fvec_L2sqr(x, c);
    - in-list scan, ``IVFFlatScanner<METRIC_L2>``: dis = fvec_L2sqr(x, y) per code vector into a k-max-heap
      (strict ``<`` against the heap top, heap order (distance, id)), results ascending by (distance, id);
      missing results are (FLT_MAX, -1);
    - f32 dot products in the structure of faiss's hand-vectorised AVX2 kernels (``fvec_L2sqr`` /
      ``fvec_norm_L2sqr``, ``distances_simd.cpp``): 8 lane accumulators over consecutive 8-float chunks
      (multiply, then add), folded to 4 lanes, a 4-float tail and a zero-padded rest added lane-wise, then
      the horizontal tree -- for d % 8 == 0 ((m4+m0) + (m5+m1)) + ((m6+m2) + (m7+m3)); the BLAS <x, c>
      uses the same structure.  A BLAS library's own summation order is implementation-defined, so
      rounding-level near-ties can still order differently under a given faiss build.
* arithmetic "exact" -- diagnostic: distances in f64, ties by (distance, id).

``blend`` is ``convert.py:353-359`` verbatim in numpy f32 semantics: weight = (1/score)^2, normalised per
row, sum over the k neighbours of big_npy[ix] * weight, then ``feats * index_rate + (1 - index_rate) * feats0``.
"""
from __future__ import annotations

import numpy as np

FLT_MAX = np.float32(np.finfo(np.float32).max)
BLAS_THRESHOLD = 20  # faiss distance_compute_blas_threshold


def _avx_sum(t):
    """faiss's AVX2 reduction of f32 terms t [..., d]: 8 lane accumulators over the whole 8-float chunks, folded
    to 4 lanes (high + low), the next 4 terms and then the zero-padded rest added lane-wise, then two hadds."""
    t = np.asarray(t, np.float32)
    d = t.shape[-1]
    n8 = d // 8 * 8
    acc = np.zeros(t.shape[:-1] + (8,), np.float32)
    for j in range(0, n8, 8):
        acc = acc + t[..., j:j + 8]
    s4 = acc[..., 4:8] + acc[..., 0:4]
    rest = t[..., n8:]
    if rest.shape[-1] >= 4:
        s4 = s4 + rest[..., :4]
        rest = rest[..., 4:]
    if rest.shape[-1]:
        pad = np.zeros(t.shape[:-1] + (4,), np.float32)
        pad[..., :rest.shape[-1]] = rest
        s4 = s4 + pad
    return (s4[..., 0] + s4[..., 1]) + (s4[..., 2] + s4[..., 3])


def fvec_l2sqr(x, y):
    """faiss fvec_L2sqr in f32: x [..., d], y [..., d] -> [...]."""
    t = np.asarray(x, np.float32) - np.asarray(y, np.float32)
    return _avx_sum(t * t)


def fvec_norm_l2sqr(x):
    x = np.asarray(x, np.float32)
    return _avx_sum(x * x)


def fvec_inner(x, y):
    return _avx_sum(np.asarray(x, np.float32) * np.asarray(y, np.float32))


def coarse_distances(q, centroids, arithmetic="faiss"):
    """[nq][nlist] squared distances of the coarse step, as the given arithmetic computes them."""
    if arithmetic == "exact":
        q64, c64 = np.asarray(q, np.float64), centroids.astype(np.float64)
        return ((q64[:, None, :] - c64[None]) ** 2).sum(-1)
    q, c = np.asarray(q, np.float32), np.asarray(centroids, np.float32)
    if len(q) >= BLAS_THRESHOLD:
        xn, cn = fvec_norm_l2sqr(q), fvec_norm_l2sqr(c)
        ip = np.stack([fvec_inner(qi[None, :], c) for qi in q])  # [nq][nlist]
        dis = (xn[:, None] + cn[None, :]) - np.float32(2) * ip
        return np.maximum(dis, np.float32(0))
    return np.stack([fvec_l2sqr(qi[None, :], c) for qi in q])


def search(index, q, k=8, nprobe=None, arithmetic="faiss"):
    """q [nq][d] f32 -> (D f32 [nq][k], I int64 [nq][k])."""
    nprobe = index.nprobe if nprobe is None else nprobe
    dc_all = coarse_distances(q, index.centroids, arithmetic)
    D = np.full((len(q), k), FLT_MAX, dtype=np.float32)
    I = np.full((len(q), k), -1, dtype=np.int64)
    for qi in range(len(q)):
        dc = dc_all[qi]
        probes = np.lexsort((np.arange(index.nlist), dc))[:nprobe]
        cand_d, cand_i = [], []
        for li in probes:
            codes = index.codes[li]
            if len(codes):
                if arithmetic == "exact":
                    cand_d.append(((codes.astype(np.float64) - np.asarray(q[qi], np.float64)) ** 2).sum(-1))
                else:
                    cand_d.append(fvec_l2sqr(codes, np.asarray(q[qi], np.float32)[None, :]).astype(np.float64))
                cand_i.append(index.ids[li])
        if cand_d:
            cd, ci = np.concatenate(cand_d), np.concatenate(cand_i)
            order = np.lexsort((ci, cd))[:k]
            D[qi, : len(order)] = cd[order].astype(np.float32)
            I[qi, : len(order)] = ci[order]
    return D, I


def blend(feats, D, I, big_npy, index_rate):
    """convert.py:353-359: feats [T][C] f32 (the tensor being blended), big_npy [ntotal][C] f32."""
    score, ix = D, I
    with np.errstate(divide="ignore", over="ignore", invalid="ignore"):
        weight = np.square(1 / score)
        npy = np.sum(big_npy[ix] * np.expand_dims(weight / weight.sum(axis=1, keepdims=True), axis=2), axis=1)
    return (npy * np.float32(index_rate) + np.float32(1 - index_rate) * feats).astype(np.float32)
