"""Device-resident FAISS IVF-Flat index and the retrieval step of ``VC.voice_conversion``
(``convert.py:349-359``): ``score, ix = index.search(feats, k=8)``; weight = (1/score)^2 normalised;
``feats = (Σ big_npy[ix] · w) · index_rate + (1 - index_rate) · feats``.

The index file is read by ``faiss_index.read_index`` (no faiss needed); centroids (transposed),
CSR inverted lists and ``big_npy = reconstruct_n(0, ntotal)`` are uploaded once.  Search and blend
are ivf.hip kernels on the channels-first [768][T_f] features, in place of the reference's
host round trip.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from .faiss_index import IVFFlatIndex, read_index


class IVFFlatDevice:
    def __init__(self, index: IVFFlatIndex, device="cuda"):
        self.d, self.nlist, self.nprobe, self.ntotal = index.d, index.nlist, index.nprobe, index.ntotal
        self.device = device
        self.centT = torch.from_numpy(np.ascontiguousarray(index.centroids.T)).to(device)
        sizes = np.array([len(i) for i in index.ids], dtype=np.int64)
        off = np.zeros(self.nlist + 1, dtype=np.int64)
        np.cumsum(sizes, out=off[1:])
        self.list_off = torch.from_numpy(off).to(device)
        codes = np.concatenate(index.codes) if off[-1] else np.zeros((1, self.d), np.float32)
        ids = np.concatenate(index.ids) if off[-1] else np.zeros(1, np.int64)
        self.codes = torch.from_numpy(np.ascontiguousarray(codes)).to(device)
        self.ids = torch.from_numpy(np.ascontiguousarray(ids)).to(device)
        self.big = torch.from_numpy(index.reconstruct_n(0, self.ntotal)).to(device)

    @classmethod
    def from_file(cls, path, device="cuda"):
        return cls(read_index(path), device)

    def search_cf(self, feats_cf, k=8, nprobe=None, arithmetic="faiss"):
        """feats_cf [d][T] device f32 (channels-first) -> (D [T][k] f32, I [T][k] int64).  ``arithmetic``:
        "faiss" = faiss's own f32 evaluation (the default; include/rvc_amd.h), "exact" = f64 (diagnostic)."""
        d, T = feats_cf.shape
        if d != self.d:
            raise ValueError(f"ivf: index dim {self.d} != features {d}")
        nprobe = self.nprobe if nprobe is None else nprobe
        D = torch.empty(T, k, device=feats_cf.device)
        I = torch.empty(T, k, dtype=torch.int64, device=feats_cf.device)
        probes = torch.empty(T, nprobe, dtype=torch.int64, device=feats_cf.device)
        ops.ivf_search(feats_cf, T, d, T, 1, self.centT, self.nlist, nprobe, self.list_off, self.codes, self.ids,
                       k, D, I, probes, {"faiss": ops.IVF_FAISS, "exact": ops.IVF_EXACT}[arithmetic])
        return D, I

    def blend_cf(self, feats_cf, D, I, index_rate):
        """convert.py:353-359 on channels-first features -> new [d][T] tensor."""
        d, T = feats_cf.shape
        out = torch.empty_like(feats_cf)
        ops.ivf_blend(feats_cf, T, d, T, 1, D, I, D.shape[1], self.big, self.ntotal, index_rate, out, T, 1)
        return out

    def retrieve_cf(self, feats_cf, index_rate, k=8):
        D, I = self.search_cf(feats_cf, k)
        return self.blend_cf(feats_cf, D, I, index_rate)
