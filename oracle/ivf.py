"""TEST INFRASTRUCTURE ONLY (parity oracle; never imported by the product path).

FAISS IVF-Flat search + the reference's retrieval blend, restated in numpy.

* ``search`` follows faiss's ``IndexIVF::search`` for an ``IndexIVFFlat`` with an ``IndexFlatL2``
  quantizer (faiss-cpu>=1.7.3, ``requirements.txt:17``; faiss itself is absent here): coarse
  assignment = the ``nprobe`` nearest centroids, then an exhaustive L2 scan of those lists keeping
  the ``k`` smallest squared distances; missing results are (FLT_MAX, -1).  Distances are exact
  (f64) and ties are broken by (distance, id) -- faiss computes in f32 (BLAS for the coarse step),
  so its order can differ from this only for near-ties within f32 rounding ("parity unpinned").
* ``blend`` is ``convert.py:353-359`` verbatim in numpy f32 semantics: weight = (1/score)^2,
  normalised per row, sum over the k neighbours of big_npy[ix] * weight, then
  ``feats * index_rate + (1 - index_rate) * feats0``.
"""
from __future__ import annotations

import numpy as np

FLT_MAX = np.float32(np.finfo(np.float32).max)


def search(index, q, k=8, nprobe=None):
    """q [nq][d] f32 -> (D f32 [nq][k], I int64 [nq][k])."""
    nprobe = index.nprobe if nprobe is None else nprobe
    q64 = np.asarray(q, dtype=np.float64)
    c64 = index.centroids.astype(np.float64)
    D = np.full((len(q), k), FLT_MAX, dtype=np.float32)
    I = np.full((len(q), k), -1, dtype=np.int64)
    for qi in range(len(q)):
        dc = ((c64 - q64[qi]) ** 2).sum(-1)  # [nlist], exact in f64
        probes = np.lexsort((np.arange(index.nlist), dc))[:nprobe]
        cand_d, cand_i = [], []
        for li in probes:
            codes = index.codes[li].astype(np.float64)
            if len(codes):
                cand_d.append(((codes - q64[qi]) ** 2).sum(-1))
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
