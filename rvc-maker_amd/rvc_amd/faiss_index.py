"""FAISS ``IndexIVFFlat`` (L2) ``.index`` files without faiss: reader, writer and the search the
reference runs (``convert.py:392-399`` read + ``reconstruct_n``; ``:349-359`` ``search(k=8)`` + blend;
built by ``create_index.py:66-83``: ``IVF{n_ivf},Flat``, L2, nprobe = 1).

faiss (``faiss-cpu>=1.7.3``, ``requirements.txt:17``) is not installed here, so the binary layout is
restated from faiss's published ``index_write.cpp`` / ``index_read.cpp`` (little-endian):

  IndexIVFFlat   fourcc "IwFl" | index header | nlist u64 | nprobe u64 | quantizer | direct map | lists
  index header   d i32 | ntotal i64 | dummy i64 (1<<20) | dummy i64 | is_trained u8 | metric i32
                 (| metric_arg f32 when metric > 1)
  quantizer      IndexFlatL2: fourcc "IxF2" | index header | n u64 | n float32 (nlist * d centroids)
  direct map     type u8 | n u64 | n int64
  lists          "ilar" | nlist u64 | code_size u64 | "full" + (n u64, nlist u64 sizes)
                 or "sprs" + (n u64, pairs (list, size)) | per non-empty list: codes, then ids (int64)

The format is therefore "parity unpinned" (no reference .index fixture exists): the round trip of
this writer/reader is tested, and the reader accepts what the writer produces and what faiss's
published writer produces for this index type.  Nothing here unpickles or executes file content.
"""
from __future__ import annotations

import io
import struct

import numpy as np

METRIC_L2 = 1


def fourcc(s: str) -> int:
    b = s.encode("ascii")
    return b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24


class IVFFlatIndex:
    """Host image of an IndexIVFFlat: centroids [nlist][d], inverted lists (codes [n][d] f32,
    ids [n] int64) and nprobe."""

    def __init__(self, d, centroids, lists_codes, lists_ids, nprobe=1, ntotal=None):
        self.d = int(d)
        self.centroids = np.ascontiguousarray(centroids, dtype=np.float32).reshape(-1, self.d)
        self.nlist = self.centroids.shape[0]
        self.codes = [np.ascontiguousarray(c, dtype=np.float32).reshape(-1, self.d) for c in lists_codes]
        self.ids = [np.ascontiguousarray(i, dtype=np.int64).reshape(-1) for i in lists_ids]
        if len(self.codes) != self.nlist or len(self.ids) != self.nlist:
            raise ValueError("IVFFlat: one code / id array per list expected")
        self.nprobe = int(nprobe)
        self.ntotal = int(ntotal) if ntotal is not None else sum(len(i) for i in self.ids)
        self.metric_type = METRIC_L2

    # -- construction for tests / tools: assign vectors to their nearest centroid (exact, f64)
    @classmethod
    def build(cls, centroids, xb, nprobe=1):
        c = np.asarray(centroids, dtype=np.float64)
        x = np.asarray(xb, dtype=np.float64)
        d2 = (x * x).sum(1)[:, None] - 2 * x @ c.T + (c * c).sum(1)[None, :]
        assign = np.argmin(d2, axis=1)
        codes, ids = [], []
        for li in range(c.shape[0]):
            sel = np.nonzero(assign == li)[0]
            codes.append(np.asarray(xb, dtype=np.float32)[sel])
            ids.append(sel.astype(np.int64))
        return cls(c.shape[1], centroids, codes, ids, nprobe=nprobe, ntotal=x.shape[0])

    def reconstruct_n(self, i0, ni):
        """IndexIVF::reconstruct_n: the stored vectors with ids in [i0, i0 + ni), in id order."""
        out = np.zeros((ni, self.d), dtype=np.float32)
        for codes, ids in zip(self.codes, self.ids):
            m = (ids >= i0) & (ids < i0 + ni)
            out[ids[m] - i0] = codes[m]
        return out

    # ------------------------------------------------------------------ binary format
    def write(self, path_or_file):
        f = io.BytesIO()
        w = f.write

        def header(d, ntotal):
            w(struct.pack("<iqqqBi", d, ntotal, 1 << 20, 1 << 20, 1, METRIC_L2))

        w(struct.pack("<I", fourcc("IwFl")))
        header(self.d, self.ntotal)
        w(struct.pack("<QQ", self.nlist, self.nprobe))
        w(struct.pack("<I", fourcc("IxF2")))
        header(self.d, self.nlist)
        w(struct.pack("<Q", self.nlist * self.d))
        w(self.centroids.astype("<f4").tobytes())
        w(struct.pack("<BQ", 0, 0))  # direct map: none, empty array
        w(struct.pack("<I", fourcc("ilar")))
        w(struct.pack("<QQ", self.nlist, self.d * 4))
        sizes = [len(i) for i in self.ids]
        if sum(1 for s in sizes if s > 0) > self.nlist // 2:
            w(struct.pack("<I", fourcc("full")))
            w(struct.pack("<Q", self.nlist))
            w(np.asarray(sizes, dtype="<u8").tobytes())
        else:
            w(struct.pack("<I", fourcc("sprs")))
            pairs = [v for li, s in enumerate(sizes) if s > 0 for v in (li, s)]
            w(struct.pack("<Q", len(pairs)))
            w(np.asarray(pairs, dtype="<u8").tobytes())
        for codes, ids in zip(self.codes, self.ids):
            if len(ids):
                w(codes.astype("<f4").tobytes())
                w(ids.astype("<i8").tobytes())
        data = f.getvalue()
        if hasattr(path_or_file, "write"):
            path_or_file.write(data)
        else:
            with open(path_or_file, "wb") as fh:
                fh.write(data)

    @classmethod
    def read(cls, path_or_bytes):
        data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
        r = _Reader(data)
        h = r.u32()
        if h not in (fourcc("IwFl"), fourcc("IvFl")):
            raise ValueError(f"read_index: not an IndexIVFFlat (fourcc {h:#x})")
        d, ntotal, metric = r.header()
        if metric != METRIC_L2:
            raise ValueError("read_index: only the L2 metric is on the path (create_index.py builds L2)")
        nlist, nprobe = r.u64(), r.u64()
        qh = r.u32()
        if qh != fourcc("IxF2"):
            raise ValueError(f"read_index: quantizer must be IndexFlatL2 (fourcc {qh:#x})")
        qd, qn, _ = r.header()
        n = r.u64()
        if qd != d or qn != nlist or n != nlist * d:
            raise ValueError("read_index: quantizer size mismatch")
        centroids = r.array("<f4", n).reshape(nlist, d)
        if h == fourcc("IwFl"):
            r.u8()  # direct map type
            r.array("<i8", r.u64())
        lh = r.u32()
        if lh != fourcc("ilar"):
            raise ValueError(f"read_index: only ArrayInvertedLists are supported (fourcc {lh:#x})")
        ln, code_size = r.u64(), r.u64()
        if ln != nlist or code_size != d * 4:
            raise ValueError("read_index: inverted-list header mismatch")
        kind = r.u32()
        sizes = np.zeros(nlist, dtype=np.int64)
        if kind == fourcc("full"):
            sizes[:] = r.array("<u8", r.u64())
        elif kind == fourcc("sprs"):
            pairs = r.array("<u8", r.u64()).reshape(-1, 2)
            sizes[pairs[:, 0].astype(np.int64)] = pairs[:, 1]
        else:
            raise ValueError(f"read_index: unknown list layout {kind:#x}")
        codes, ids = [], []
        for s in sizes:
            s = int(s)
            codes.append(r.array("<f4", s * d).reshape(s, d) if s else np.zeros((0, d), np.float32))
            ids.append(r.array("<i8", s) if s else np.zeros(0, np.int64))
        return cls(d, centroids, codes, ids, nprobe=nprobe, ntotal=ntotal)


class _Reader:
    def __init__(self, data):
        self.b = memoryview(data)
        self.o = 0

    def take(self, n):
        if self.o + n > len(self.b):
            raise ValueError("read_index: truncated file")
        v = self.b[self.o: self.o + n]
        self.o += n
        return v

    def u8(self):
        return struct.unpack("<B", self.take(1))[0]

    def u32(self):
        return struct.unpack("<I", self.take(4))[0]

    def u64(self):
        return struct.unpack("<Q", self.take(8))[0]

    def header(self):
        d, ntotal, _, _, _trained, metric = struct.unpack("<iqqqBi", self.take(4 + 8 * 3 + 1 + 4))
        if metric > 1:
            self.take(4)
        return d, ntotal, metric

    def array(self, dt, n):
        n = int(n)
        return np.frombuffer(self.take(n * np.dtype(dt).itemsize), dtype=dt).astype(dt[1:], copy=True)


def read_index(path):
    """``faiss.read_index`` for the IVF-Flat indexes ``create_index.py`` writes."""
    return IVFFlatIndex.read(path)
