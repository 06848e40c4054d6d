"""Bench: end-to-end VC (ContentVec + RMVPE + TextEncoder/flow/NSF-HiFiGAN), 48k v2, one 30 s clip
per GPU per step (BASELINE.json configs[1]; N>1 = configs[3]-style utterance sharding with the
output waveforms gathered to rank 0 over RCCL).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--seconds S] [--no-cpu-baseline] [--no-stream]
    python bench.py --gpus N --utterances 120 --seconds 30     # BASELINE configs[3]: 1 h over N GPUs

Default: a clip stream (VC.pipeline_device_stream) -- K steps are K clips per GPU, clip k+1's front end
(filtfilt, RMVPE, ContentVec) running on its own streams under clip k's synthesizer; the line also carries
"per_call", the same K clips as one finished pipeline_device call each.  Each clip's output waveform is copied
to pinned host memory inside the timed region (host-visible output; --hbm-output leaves it in HBM).

--utterances U (BASELINE configs[3], SURVEY §8(d) cfg 4): a fixed job of U utterances of --seconds each (1 h =
120 x 30 s), sharded longest-first over the ranks (rvc_amd.shard.shard_utterances), each rank's share issued as
one clip stream, the output waveforms gathered to rank 0 by grouped send / recv (RCCL over xGMI); a step is the
whole job, "scaling": "strong".  Utterance i draws its noise with seed 17 + i (shard.convert_utterances), so the
gathered waveforms are the same bits at every world size (tests/test_gpu_shard.py).

--gpus N without WORLD_SIZE in the environment starts N ranks itself (torch.distributed.run as a
child process, one rank per GPU); under an external launcher WORLD_SIZE must equal N.

Prints ONE JSON line on rank 0 (contract in the task statement): metric/value = output
audio-seconds per wall-second for the whole job, plus "roofline" for the dominant kernel
family (the split-operand MFMA conv engine: conv_x6_kernel + the fused ResBlock pairs; algorithmic FLOPs over the
device's own kernel stamps of one instrumented per-call pass, torch.profiler, with the HIP-event time beside it),
its "families" (attention -- split-fp16 or f32 MFMA --, the BiGRU's us per step against its hand-off floor, and the HBM GB/s of
LayerNorm / fe0 / STFT / filtfilt), and "cpu_baseline" (the torch-CPU oracle on a bounded clip, rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "audio-seconds/sec/GPU (xRT) end-to-end VC, 48k v2; 1/2/4/8 GPU scaling"
PEAK_F32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32 MFMA dense peak (= f32 vector peak)
PEAK_MFMA16_TFLOPS = 2500.0  # bf16 / fp16 dense MFMA peak (MI355X_MICROARCH.md)
PEAK_F64_MFMA_TFLOPS = 78.6  # MI355X f64 matrix peak (AMD spec; the f64 RMVPE's conv engine, rmvpe64.hip)
F64_MEASURED_TFLOPS = 39.0  # the MFMA-only f64 loop on every CU, real operands (scripts/conv64_dbg.hip, round 4)


def pass_peak(passes):
    """The f32-equivalent ceiling of one split-operand launch: the 16-bit dense MFMA peak over the MFMA passes
    each product takes (6 / 8 split-bf16, 3 split-fp16 or bf16x3, 1 bf16)."""
    n = {16: 3, 7: 6}.get(passes, passes)  # RVC_ARITH_F16X3: 3 fp16 passes; RVC_ARITH_FP32_SA: 6 passes
    return PEAK_MFMA16_TFLOPS / n
DTYPES = {"fp32": "f32-equivalent (split-fp16 3-pass MFMA for the generator's convs -- scale from the producer's "
                  "published |max| -- and ResBlock pairs, split-bf16 6-pass MFMA elsewhere; f32 accumulate; RMVPE f64 "
                  "with its GRU recurrence f32)",
          "fp32x6": "f32 (split-bf16 x6 MFMA, f32 accumulate)",
          "f16x3": "f32-equivalent (split-fp16 3-pass MFMA convs, power-of-2 scaled 22-bit operands, f32 accumulate)",
          "bf16x3": "bf16x3 (3-pass split-bf16 MFMA convs, f32 accumulate; f32 elsewhere)",
          "bf16": "bf16 (bf16-operand MFMA convs, f32 accumulate; f32 elsewhere)"}


def build_models(dev, sr=48000, version="v2", seed=1234):
    from rvc_amd import synthetic
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(sr, version, seed=seed), dev)
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(seed + 1), dev)
    vc = VC(sr, Config(dev), rmvpe=RMVPEAMD(synthetic.rmvpe_state_dict(seed + 2), dev))
    return vc, hub, net_g


class ConvProbe:
    """Wraps ops.conv1d and ops.resblock_pair during one instrumented step: HIP events around every
    launch on the launch stream + the launch's algorithmic FLOPs (reference conv FLOPs) +
    its engine (a fused ResBlock pair counts as split-bf16 work: its two convs' FLOPs)."""

    def __init__(self):
        from rvc_amd import ops
        self.ops = ops
        self.orig = ops.conv1d
        self.orig_rb = ops.resblock_pair
        self.orig_64 = ops.conv64
        self.orig_w64 = ops.wino64
        self.rec = []
        self.aux = []  # (family, algorithmic FLOPs, algorithmic HBM bytes, frames) of the non-conv kernels (families())

    def __enter__(self):
        import ctypes
        from rvc_amd import _lib
        lib = _lib.load()

        def wrapped(*a, **k):
            # e0 before the call; em is recorded by the library right after the conv kernel, before its split-K
            # reduce (rvc_conv1d_set_probe_event), so e0 -> em brackets the conv kernel alone
            s = torch.cuda.current_stream()
            e0, em = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            em.record(s)  # creates the event's handle (the library records it again after the kernel)
            e0.record(s)
            lib.rvc_conv1d_set_probe_event(ctypes.c_void_p(em.cuda_event))
            try:
                out = self.orig(*a, **k)
            finally:
                lib.rvc_conv1d_set_probe_event(None)
            self.rec.append((e0, em, self.ops.LAST_CONV_FLOPS, self.ops.LAST_CONV_ENGINE, self._bytes(a, k, out),
                             self.ops.LAST_CONV_PASSES))
            return out
        def wrapped_rb(x, y, c1, c2, dil, slope, accumulate=False):
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            out = self.orig_rb(x, y, c1, c2, dil, slope, accumulate=accumulate)
            e1.record(s)
            B = x.shape[0] if x.dim() == 3 else 1  # the synthesizer passes [B][C][L] since it batches clips
            C, L = x.shape[-2], x.shape[-1]
            flops = 2 * 2.0 * B * C * C * c1.K * L
            nbytes = 4.0 * (B * C * L * (2 + bool(accumulate)) + 2 * C * C * c1.K)  # x, y (+ y read), both weights
            self.rec.append((e0, e1, flops, 1, nbytes, self.ops.rb_passes(c1.K)))
            return out
        def wrapped_64(x, w, Ci, Co, K, **k):
            # the f64 RMVPE's convs (engine 2): events around the call (its split-K reduce included)
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            out = self.orig_64(x, w, Ci, Co, K, **k)
            e1.record(s)
            B = k.get("B") or (1 if x.dim() == 2 else x.shape[0])
            Lout, wrap = out.shape[-1] if k.get("Lout") is None else k["Lout"], k.get("wrap", 0)
            valid = (Lout // wrap - 2) * (wrap - 2) if wrap else Lout
            self.rec.append((e0, e1, 2.0 * B * Co * Ci * K * valid, 2, 0.0, 64))
            return out
        def wrapped_w64(x, v, Ci, Co, H, W, **k):
            # the f64 RMVPE's Winograd convs (engine 2): the ALGORITHMIC FLOPs of the direct 3x3 conv they replace
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            out = self.orig_w64(x, v, Ci, Co, H, W, **k)
            e1.record(s)
            self.rec.append((e0, e1, 2.0 * k.get("B", 1) * Co * Ci * 9 * H * W, 2, 0.0, 64))
            return out
        self.ops.conv1d = wrapped
        self.ops.resblock_pair = wrapped_rb
        self.ops.conv64 = wrapped_64
        self.ops.wino64 = wrapped_w64
        # the other kernel families of the pass (roofline "families"): algorithmic work per call, timed by the
        # profiler pass (their device stamps); no events around them
        ops = self.ops
        self.saved = {n: getattr(ops, n) for n in ("attention", "layernorm_cf", "fe0_gn_gelu", "bigru64_batched",
                                                   "stft_mag64")}
        self.saved_filt = ops.FiltFilt.__call__
        aux = self.aux

        def attention(q, k, v, o, *, B, H, D, T, **kw):
            # softmax(Q K^T) V: 4 T^2 D FLOP per head (the reference's dense scores and PV); the relative band (rk, ev:
            # the TextEncoder) adds 2 * 2 T (2W + 1) D; bytes: q, k, v read and o written once
            fl = 4.0 * B * H * T * T * D + (4.0 * B * H * T * (2 * kw.get("W", 0) + 1) * D if kw.get("rk") is not None
                                            else 0.0)
            aux.append(("attention_d%d" % D, fl, 4.0 * 4 * B * H * D * T, T))
            return self.saved["attention"](q, k, v, o, B=B, H=H, D=D, T=T, **kw)

        def layernorm_cf(x, res, gamma, beta, out, B, C, T, *a, **kw):
            aux.append(("layernorm", 0.0, 4.0 * B * C * T * (2 + (res is not None)), T))
            return self.saved["layernorm_cf"](x, res, gamma, beta, out, B, C, T, *a, **kw)

        def fe0_gn_gelu(wav, w_km, gamma, beta, B, N, C, K, stride, *a, **kw):
            T = (N - K) // stride + 1
            # the conv twice (statistics, then apply) over the signal; bytes: the signal (twice) and the output once
            aux.append(("fe0", 2 * 2.0 * B * C * K * T, 4.0 * B * (2 * N + C * T), T))
            return self.saved["fe0_gn_gelu"](wav, w_km, gamma, beta, B, N, C, K, stride, *a, **kw)

        def bigru64_batched(gi, whh, bhh, y, gran, err, B, T):
            aux.append(("bigru", 0.0, 8.0 * B * (1536 + 512) * T, T))
            return self.saved["bigru64_batched"](gi, whh, bhh, y, gran, err, B, T)

        def stft_mag64(x, win, mag, N, F, nfft, hop):
            aux.append(("stft", 0.0, 4.0 * N + 8.0 * F * (nfft // 2 + 1), F))
            return self.saved["stft_mag64"](x, win, mag, N, F, nfft, hop)

        def filt_call(fself, x, tpad, want_f64=False):
            N = x.numel()
            aux.append(("filtfilt", 0.0, 4.0 * N + 4.0 * (N + 2 * tpad) + (8.0 * (N + 2 * tpad) if want_f64 else 0), N))
            return self.saved_filt(fself, x, tpad, want_f64)

        for n, f in (("attention", attention), ("layernorm_cf", layernorm_cf), ("fe0_gn_gelu", fe0_gn_gelu),
                     ("bigru64_batched", bigru64_batched), ("stft_mag64", stft_mag64)):
            setattr(ops, n, f)
        ops.FiltFilt.__call__ = filt_call
        return self

    def __exit__(self, *exc):
        self.ops.conv1d = self.orig
        self.ops.resblock_pair = self.orig_rb
        self.ops.conv64 = self.orig_64
        self.ops.wino64 = self.orig_w64
        for n, f in self.saved.items():
            setattr(self.ops, n, f)
        self.ops.FiltFilt.__call__ = self.saved_filt

    @staticmethod
    def _bytes(a, k, out):
        """Algorithmic HBM bytes of one conv launch: input once, f32 weights once, output written,
        residual / accumulate operands read once."""
        x, Ci, Co, K = a[0], a[2], a[3], a[4]
        B = k.get("B") or (1 if x.dim() == 2 else x.shape[0])
        Lin = k.get("Lin") or x.shape[-1]
        groups, nphase = k.get("groups", 1), k.get("nphase", 1)
        n_out = out.numel() if k.get("out") is None else B * Co * (k.get("Lout") or out.shape[-1])
        reads = B * Ci * Lin + nphase * (Ci // groups) * K * Co
        reads += n_out * ((k.get("res") is not None) + bool(k.get("accumulate")))
        return 4.0 * (reads + n_out)

    def summary(self, engine=None):
        """(launches, kernel ms, algorithmic FLOPs) over the launches of one engine (None = all)."""
        torch.cuda.synchronize()
        rec = [r for r in self.rec if engine is None or r[3] == engine]
        ms = [r[0].elapsed_time(r[1]) for r in rec]
        fl = [r[2] for r in rec]
        return len(ms), float(sum(ms)), float(sum(fl))

    def by_passes(self):
        """Split-operand launches grouped by pass set: {passes: (launches, kernel ms, FLOPs)}, and the
        FLOP-weighted ceiling of the family: sum FLOPs / sum (FLOPs / the launch's own pass-set peak)."""
        torch.cuda.synchronize()
        groups = {}
        for r in self.rec:
            if r[3] != 1:
                continue
            g = groups.setdefault(r[5], [0, 0.0, 0.0])
            g[0] += 1
            g[1] += r[0].elapsed_time(r[1])
            g[2] += r[2]
        tot = sum(g[2] for g in groups.values())
        weighted = tot / sum(g[2] / pass_peak(p) for p, g in groups.items()) if tot else None
        return groups, weighted

    def algorithmic_bytes(self, engine=None):
        rec = [r for r in self.rec if engine is None or r[3] == engine]
        return float(sum(r[4] for r in rec)) / max(len(rec), 1)


def _pass_set(name):
    """The pass set of a split-operand kernel from its template arguments (conv_x6_kernel<FM, FN, WM, WN, NI, NP,
    F16, SA>, resblock_x6_kernel<C, NP, F16>), in ConvProbe's keys: 16 = split-fp16, 7 = split accumulators."""
    args = [t.strip() for t in name.split("<", 1)[1].split(">", 1)[0].split(",")]
    if name.startswith("conv_x6_kernel"):
        np_, f16, sa = int(args[5]), args[6] == "true", args[7] == "true"
    else:
        np_, f16, sa = int(args[1]), args[2] == "true", False
    return 16 if f16 else (7 if sa else np_)


# kernel families beside the split-operand conv engine (the roofline's "families"): name prefix -> family
FAMILY_KERNELS = (("attn_fwd_kernel<64>", "attention_d64"), ("attn_combine_kernel<64>", "attention_d64"),
                  ("attn_f16_kernel<64>", "attention_d64"), ("attn_f16_kernel<96>", "attention_d96"),
                  ("attn_fwd_kernel<96>", "attention_d96"), ("attn_combine_kernel<96>", "attention_d96"),
                  ("attn_relv_band_kernel", "attention_d96"), ("bigru", "bigru"), ("layernorm_cf", "layernorm"),
                  ("fe0_", "fe0"), ("filt_", "filtfilt"), ("stft_mag_kernel", "stft"))
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s
# the BiGRU step's hand-off floor: the fastest step measured for this exchange (both directions
# XCD-local, f32 recurrence, 1.43 us alone) -- the device-coherent granule round trip every step pays
BIGRU_FLOOR_US = 1.43


def profiler_kernel_times(fn, families=None):
    """{pass set: (launches, device ms)} of the split-operand kernels one call of ``fn`` launches, from
    torch.profiler's device records; None when the profiler is unavailable (or rocprofv3 already traces).
    ``families`` (a dict) receives {family: [launches, device ms, matched prefixes]} of the FAMILY_KERNELS of the same
    call."""
    if "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ):
        return None
    try:
        from torch.profiler import ProfilerActivity, profile
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            fn()
            torch.cuda.synchronize()
        out = {}
        for e in prof.events():
            name = e.name.replace("(anonymous namespace)::", "").replace("void ", "")
            if families is not None:
                for pre, fam in FAMILY_KERNELS:
                    if name.startswith(pre):
                        g = families.setdefault(fam, [0, 0.0, set()])
                        g[0] += 1
                        g[1] += e.time_range.elapsed_us() * 1e-3
                        g[2].add(pre)
                        break
            if not (name.startswith("conv_x6_kernel<") or name.startswith("resblock_x6_kernel<")):
                continue
            g = out.setdefault(_pass_set(name), [0, 0.0])
            g[0] += 1
            g[1] += e.time_range.elapsed_us() * 1e-3
        return out or None
    except Exception as exc:  # noqa: BLE001 -- a missing tracer leaves the event timing in place
        print(f"bench.py: torch.profiler unavailable ({exc}); roofline from HIP events", file=sys.stderr)
        return None


def family_rooflines(aux, fam_ms):
    """The roofline entries of the kernel families beside the conv engine, from one pass: algorithmic work per family
    (ConvProbe.aux) over its device kernel time (profiler_kernel_times' families)."""
    tot = {}
    for fam, fl, by, T in aux:
        t = tot.setdefault(fam, [0.0, 0.0, 0, 0])
        t[0] += fl
        t[1] += by
        t[2] += 1
        t[3] += T
    out = {}
    for fam, (fl, by, calls, T) in sorted(tot.items()):
        if fam not in fam_ms:
            continue
        n, ms, kinds = fam_ms[fam]
        e = {"calls": calls, "launches": n, "kernel_ms": round(ms, 4)}
        if fam.startswith("attention"):
            tf = fl / (ms * 1e-3) / 1e12
            # split-fp16 (attn_f16_kernel, round 6): 3 fp16 MFMA passes per product -> 2.5 PF / 3 f32-equivalent
            f16 = any(k.startswith("attn_f16") for k in kinds)
            peak = PEAK_MFMA16_TFLOPS / 3 if f16 else PEAK_F32_MFMA_TFLOPS
            engine = ("split-fp16 flash attention (hH + hL + lH on v_mfma_f32_16x16x32_f16, scales from the QKV "
                      "projection's |max| cell; peak = 2.5 PF / 3)" if f16 else
                      "flash attention on the f32 MFMA (v_mfma_f32_16x16x4_f32), split-KV + combine")
            e.update(bound="mfma", achieved=round(tf, 2), peak=round(peak, 1), unit="TFLOP/s",
                     frac=round(tf / peak, 4), gflop=round(fl / 1e9, 2),
                     kernel=("ContentVec MHA 12 x 64 (fairseq.py:355)" if fam == "attention_d64" else
                             "TextEncoder rel-pos MHA 2 x 96, window 10, + its rel-v band kernel (synthesizers.py:227-251)")
                     + ": " + engine + "; FLOPs = 4 T^2 D per head (+ the relative band)")
        elif fam == "bigru":
            us = ms * 1e3 / max(T, 1)
            e.update(bound="latency", unit="us/step", achieved=round(us, 3), floor=BIGRU_FLOOR_US,
                     frac=round(BIGRU_FLOOR_US / us, 4), steps=T,
                     kernel="RMVPE BiGRU recurrence (RMVPE.py:254-260): 16 workgroups per direction, one device-"
                            "coherent granule hand-off per step; floor = the fastest measured step of this exchange "
                            "(DESIGN.md §7), frac = floor / achieved")
        else:
            gbs = by / (ms * 1e-3) / 1e9
            e.update(bound="latency (sequential IIR)" if fam == "filtfilt" else "hbm", unit="GB/s",
                     achieved=round(gbs, 1), peak=HBM_PEAK_GBS, frac=round(gbs / HBM_PEAK_GBS, 4),
                     algorithmic_mb=round(by / 1e6, 2))
        out[fam] = e
    return out


def park_gpu(seconds):
    """Occupy the current stream for about ``seconds`` with torch's spin kernel (calibrated once)."""
    global _SLEEP_RATE
    if _SLEEP_RATE is None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.cuda._sleep(1 << 22)
        e1.record()
        torch.cuda.synchronize()
        _SLEEP_RATE = (1 << 22) / max(e0.elapsed_time(e1) * 1e-3, 1e-6)  # cycles per second
    torch.cuda._sleep(int(_SLEEP_RATE * seconds))
_SLEEP_RATE = None


def kernel_source_hash():
    """sha256 over the library's sources (rvc-maker_amd/csrc/*.hip|cpp|h, include/*.h): the tree a PMC summary was
    measured on (scripts/pmc_traffic.py stamps it)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(REPO, "rvc-maker_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(REPO, "rvc-maker_amd", "csrc", "*.cpp")) +
                   glob.glob(os.path.join(REPO, "rvc-maker_amd", "csrc", "*.h")) +
                   glob.glob(os.path.join(REPO, "include", "*.h")))
    for fn in files:
        h.update(os.path.relpath(fn, REPO).encode())
        with open(fn, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel_family="x6"):
    """Per-launch HBM bytes of a conv family from the newest committed PMC summary of this same bench step
    (scripts/pmc_traffic.sh: separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes, FETCH_SIZE doubled per
    MI355X_MICROARCH.md) -- only when it was measured on these kernel sources (its "source_hash" equals
    kernel_source_hash()); otherwise (None, reason)."""
    import glob
    names = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_traffic.json")), reverse=True)
    for fn in names:
        try:
            with open(fn) as f:
                d = json.load(f)
            val = d[kernel_family]["traffic_bytes_per_launch"]
        except (OSError, KeyError, ValueError):
            continue
        src = d.get("source_hash")
        if src != kernel_source_hash():
            return None, f"{os.path.basename(fn)} was measured on kernel sources {src}, not this tree's " \
                         f"{kernel_source_hash()}: traffic not re-measured"
        return val, os.path.basename(fn)
    return None, "no PMC summary committed"


def synthetic_ivf(dev, n=100_000, nlist=2564, seed=77):
    """SURVEY §8(d) cfg 3 index shape as a host IVFFlatIndex: IVF2564,Flat over 100k 768-d vectors, nprobe 1.
    Vectors are drawn around 2564 seeded centres (a trained IVF index has balanced lists; uniform Gaussians in
    768-d would pile most vectors onto a few "hub" centroids); the centres are the IVF centroids.  The list
    assignment (nearest centre) runs on ``dev`` (host-side index build, never timed)."""
    from rvc_amd.faiss_index import IVFFlatIndex
    rng = np.random.default_rng(seed)
    cent = rng.standard_normal((nlist, 768)).astype(np.float32)
    xb = (cent[rng.integers(0, nlist, n)] + 0.35 * rng.standard_normal((n, 768))).astype(np.float32)
    x = torch.from_numpy(xb).to(dev)
    c = torch.from_numpy(cent).to(dev)
    assign = torch.cdist(x, c).argmin(1).cpu().numpy()
    order = np.argsort(assign, kind="stable")
    sizes = np.bincount(assign, minlength=nlist)
    off = np.concatenate([[0], np.cumsum(sizes)])
    codes = [xb[order[off[i]:off[i + 1]]] for i in range(nlist)]
    ids = [order[off[i]:off[i + 1]].astype(np.int64) for i in range(nlist)]
    return IVFFlatIndex(768, cent, codes, ids, nprobe=1, ntotal=n)


def synthetic_index(dev, n=100_000, nlist=2564, seed=77):
    """synthetic_ivf uploaded to the device (retrieval.IVFFlatDevice)."""
    from rvc_amd.retrieval import IVFFlatDevice
    return IVFFlatDevice(synthetic_ivf(dev, n, nlist, seed), dev)


def cpu_calibration():
    """Oracle-vs-reference CPU timing ratio measured in the build container (scripts/cpu_calibrate.py:
    the reference's own VC.pipeline and oracle.pipeline on the same clip, same threads), or None."""
    try:
        with open(os.path.join(REPO, "profiles", "cpu_calibration.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def cpu_threads():
    """The torch thread count the committed host scan (scripts/cpu_threads.py -> profiles/*cpu_threads.json)
    measured fastest on the GPU box's CPU share, or None (torch's default, OMP_NUM_THREADS)."""
    import glob
    for fn in sorted(glob.glob(os.path.join(REPO, "profiles", "*cpu_threads.json")), reverse=True):
        try:
            with open(fn) as f:
                return int(json.load(f)["best_threads"]), os.path.basename(fn)
        except (OSError, KeyError, ValueError):
            continue
    return None, None


def cpu_baseline(seconds=30.0):
    """The torch-CPU oracle (a restatement of the reference's CPU path) on the config's own clip length
    (30 s, ~15-20 s of CPU work on the GPU box's host threads), at the thread count the committed scan found
    fastest (cpu_threads)."""
    best, scan = cpu_threads()
    if best:
        torch.set_num_threads(best)
    from oracle import contentvec as ocv
    from oracle import pipeline as opl
    from oracle import rmvpe as orm
    from oracle import synth as osy
    from rvc_amd import melbasis, synthetic
    seed = 1234
    ck = synthetic.make_synth_ckpt(48000, "v2", seed=seed)
    Ws, Wc = osy.load_weights(ck["weight"]), ocv.load_weights(synthetic.make_contentvec_ckpt(seed + 1))
    Wr = orm.load_weights(synthetic.rmvpe_state_dict(seed + 2))
    mb = torch.from_numpy(melbasis.mel_filterbank())
    audio = synthetic.synthetic_audio(seconds, seed=1000)
    g = torch.Generator().manual_seed(0)
    noise = lambda s, k, sh: torch.randn(*sh, generator=g)  # noqa: E731
    t0 = time.perf_counter()
    out = opl.pipeline(Wc, Ws, Wr, mb, ck["config"], 0, audio, 0.0, "v2", 0.33, noise)
    dt = time.perf_counter() - t0
    cal = cpu_calibration()
    return {"value": round(len(out) / 48000 / dt, 4), "unit": "audio-s/s", "cores": torch.get_num_threads(),
            "host_cpus": os.cpu_count(), "kind": "port",
            "sample": f"{seconds:g} s clip, 48k v2, RMVPE, fp32, torch-CPU oracle (oracle/), wall {dt:.2f} s, "
                      f"{torch.get_num_threads()} torch threads ("
                      + (f"the fastest of the host scan profiles/{scan}; " if best else "")
                      + f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}: the host's CPU share for "
                      f"this GPU; os.cpu_count() = {os.cpu_count()} counts every GPU's share)",
            "oracle_over_reference_time": cal.get("oracle_over_reference_time") if cal else None,
            "calibration": (f"oracle / reference wall time on one {cal['seconds']:g} s clip in the build container "
                            f"({cal['threads']} threads): {cal['oracle_s']:.2f} s / {cal['reference_s']:.2f} s "
                            "(profiles/cpu_calibration.json)") if cal else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 12 clips per timed stream (round 6; 5 before): the stream's fill -- clip 1's front end with nothing under it, the
    # last clip's synthesizer alone -- is ~11 ms, so the value grows with K (one box, r6h: 1013 xRT at 5 clips, 1053-1064
    # at 12); 12 x 30 s clips still time in ~0.35 s
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-call", action="store_true", help="skip the per-call comparison after a clip stream")
    ap.add_argument("--no-roofline", action="store_true", help="skip the instrumented roofline pass (profiling)")
    # variants beyond the headline config (BASELINE configs 3/5 ingredients); defaults = configs[1]
    ap.add_argument("--sr", type=int, default=48000, choices=[32000, 40000, 48000])
    ap.add_argument("--f0", default="rmvpe", help="rmvpe | crepe-{tiny,small,medium,large,full} | pm")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp32x6", "f16x3", "bf16x3", "bf16"],
                    help="split-bf16 conv engine arithmetic: 6 / 3 / 1 bf16 MFMA passes per product")
    ap.add_argument("--chunks", type=int, default=1,
                    help="clips per GPU per step (BASELINE configs[2]: 64 x 10 s chunks; each a distinct clip)")
    ap.add_argument("--batch", type=int, default=1,
                    help="clips per batched pass (VC.pipeline_device_batch: RMVPE + ContentVec batched over equal-"
                         "length clips); --chunks must be a multiple")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as one hipGraph per clip (rvc_amd.graph.ClipGraph, BASELINE configs[4])")
    ap.add_argument("--no-stream", dest="stream", action="store_false",
                    help="per-call passes (one VC.pipeline_device per clip, each finished before the next) instead of "
                         "the default clip stream (VC.pipeline_device_stream: clip k+1's filtfilt / f0 / features on "
                         "a front stream while clip k's synthesizer runs on a back stream; K steps = K clips per GPU, "
                         "all issued inside the timed region)")
    ap.add_argument("--utterances", type=int, default=0,
                    help="> 0: BASELINE configs[3] -- a fixed job of U utterances sharded over the ranks (strong "
                         "scaling; a step = the whole job)")
    ap.add_argument("--hbm-output", action="store_true",
                    help="leave each output waveform in HBM (no per-clip D2H copy to pinned host memory in the timed "
                         "region; the default copies each clip's waveform to the host as VC.pipeline's .cpu() does)")
    ap.add_argument("--index-rate", type=float, default=0.0,
                    help="> 0: FAISS IVF-Flat retrieval over a synthetic index (SURVEY §8d cfg 3 shape)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launcher: start one rank per GPU under torch.distributed.run as a CHILD process and exit with
        # its code.  This process never touches the GPU (no exec after GPU init).
        return launch_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU")
    ndev = torch.cuda.device_count()
    dev_idx = local % max(ndev, 1)
    # ranks sharing a device (a rehearsal on a box with fewer GPUs than ranks) cannot use RCCL between
    # them: the gather then runs over gloo through host memory, and the line says so
    shared = world > ndev
    backend = "gloo" if shared else "nccl"
    dist = None
    torch.cuda.set_device(dev_idx)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev_idx}"))
        else:
            dist.init_process_group("gloo")
    dev = f"cuda:{dev_idx}"

    from rvc_amd import ops, synthetic
    from rvc_amd.shard import gather_waveforms
    ops.set_precision(args.precision)
    vc, hub, net_g = build_models(dev, sr=args.sr)
    index = None
    if args.index_rate > 0:
        index = synthetic_index(dev)
    if args.f0.startswith("crepe-"):
        from rvc_amd.crepe import CrepeAMD
        cap = args.f0.split("-", 1)[1]
        vc.crepe[cap] = CrepeAMD(synthetic.crepe_state_dict(1240, cap), cap, dev)
    # inputs resident in HBM before the timed region: one distinct clip per chunk
    mine = shards = None
    if args.utterances > 0:  # cfg 4: this rank's share of the whole job (input seed = 1000 + utterance index, §8(d))
        from rvc_amd.shard import shard_utterances
        if args.graph or args.batch > 1 or args.chunks > 1:
            raise SystemExit("bench.py: --utterances runs the clip stream (no --graph / --batch / --chunks)")
        shards = shard_utterances([int(args.seconds * 16000)] * args.utterances, world)
        mine = shards[rank]
        clips = [torch.from_numpy(synthetic.synthetic_audio(args.seconds, seed=1000 + i)).to(dev) for i in mine]
        args.stream = True
    else:
        clips = [torch.from_numpy(synthetic.synthetic_audio(args.seconds, seed=1000 + 97 * rank + c)).to(dev)
                 for c in range(max(1, args.chunks))]
    audio_dev = clips[0] if clips else None
    # noise seeds: clip k of a rank's stream draws seed vc.seed + k; ranks start far apart so no two clips of the
    # job share noise (cfg 4 keys each utterance's seed to its global index instead: shard.convert_utterances)
    vc.seed = 17 + 1_000_003 * rank
    host_visible = not args.hbm_output and mine is None
    out_cap = int(args.seconds * args.sr) + args.sr  # >= one clip's output samples
    host_bufs = []

    def host_buffers(n):
        """n pinned host buffers for the clips' waveforms (the reference signature's .cpu(), convert.py:455)."""
        while len(host_bufs) < n:
            host_bufs.append(torch.empty(out_cap, dtype=torch.float32, pin_memory=True))
        return host_bufs[:n]

    clip_graph = None
    if args.graph:
        from rvc_amd.graph import ClipGraph
        clip_graph = ClipGraph(vc, hub, net_g, 0, audio_dev.numel(), 0, "v2", 0.33, index, args.index_rate, args.f0)

    if args.graph:
        args.stream = False  # the graph replays are their own chunk loop
    if args.batch > 1 and (args.graph or (not args.stream and len(clips) % args.batch)):
        raise SystemExit("bench.py: --batch needs eager mode, and --chunks a multiple of it without the clip stream")

    def step():
        outs = []
        if args.batch > 1:
            for g0 in range(0, len(clips), args.batch):
                outs += vc.pipeline_device_batch(hub, net_g, 0, clips[g0:g0 + args.batch], 0, "v2", 0.33, index,
                                                 args.index_rate, args.f0)
            clips_iter = []
        else:
            clips_iter = clips
        for clip in clips_iter:
            if clip_graph is not None:
                outs.append(clip_graph(clip).clone() if len(clips) > 1 else clip_graph(clip))
            else:
                outs.append(vc.pipeline_device(hub, net_g, 0, clip, 0, "v2", 0.33, index, args.index_rate, args.f0))
        if host_visible:  # each waveform to pinned host memory, as VC.pipeline hands it back
            for o, hb in zip(outs, host_buffers(len(outs))):
                hb[: o.numel()].copy_(o, non_blocking=True)
        if dist is not None:
            # the path's only collective: output waveforms gathered to rank 0 (RCCL over xGMI)
            got = gather_waveforms(outs, dist, dst=0)
            if got is not None:
                gathered[0] += sum(len(g) for g in got)
        return outs[-1]

    def run_stream(nsteps):
        # one stream over nsteps x chunks clips: every clip's whole pass is issued inside the call, and the
        # call returns after the last clip's output is ordered on this stream
        if mine is not None:  # cfg 4: a step is the whole job -- this rank's utterances, then the gather
            from rvc_amd.shard import convert_utterances
            last = None
            for _ in range(nsteps):
                got = convert_utterances(vc, hub, net_g, 0, clips, shards, dist, 0, "v2", 0.33, index, args.index_rate,
                                         args.f0, seed=17, stats=p2p)
                if dist is not None and got is not None:
                    gathered[0] += len(got)
                last = got[-1] if got else last
            return last
        order = [clips[i % len(clips)] for i in range(nsteps * len(clips))]
        outs = vc.pipeline_device_stream(hub, net_g, 0, order, 0, "v2", 0.33, index, args.index_rate, args.f0,
                                         batch=args.batch, host_out=host_buffers(len(order)) if host_visible else None)
        if dist is not None:
            got = gather_waveforms(outs, dist, dst=0)
            if got is not None:
                gathered[0] += sum(len(g) for g in got)
        return outs[-1]

    p2p = {}

    gathered = [0]
    if host_visible:  # pinned buffers allocated before the timed region
        host_buffers(max(args.steps, args.warmup, 1) * len(clips))

    if args.stream:
        if args.warmup:
            run_stream(args.warmup)
    else:
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.stream:
        out = run_stream(args.steps)
    for _ in range(0 if args.stream else args.steps):
        out = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    vc.check_errors()  # device-side failure flags (BiGRU hand-off timeout) -- raises instead of a number
    if dist is not None:
        t = torch.tensor([dt], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    per_call = None
    if args.stream and world == 1 and not args.no_per_call and mine is None:
        # the same K steps as one pipeline_device call per clip, each finished before the next (the
        # reference's loop): the stream's gain over it, measured on the same box right after
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dt1 = time.perf_counter() - t1
        per_call = {"value": round(args.steps * len(clips) * (out.numel() / float(args.sr)) / dt1, 3),
                    "ms_per_step": round(dt1 / args.steps * 1e3, 3)}
    # every clip has the same length (a cfg-4 rank with no utterances has no output of its own)
    audio_s = out.numel() / float(args.sr) if out is not None else 0.0  # (only rank 0, which has one, prints)
    if mine is not None:  # cfg 4: the whole job's audio over the max-over-ranks time (strong scaling)
        value = args.steps * args.utterances * audio_s / dt
    else:
        value = world * args.steps * len(clips) * audio_s / dt  # whole job: every rank's clips over the max time
    gathered_per_step = gathered[0] / max(args.warmup + args.steps, 1) if dist is not None else len(clips)

    roof = None
    if rank == 0 and not args.no_roofline and mine is None:
        with ConvProbe() as probe:  # one eager pass (a graph replay launches no host-side conv calls)
            # park the GPU first so that the host queues the pass's launches ahead of it: each event pair then
            # brackets its kernel, not the host's issue gap before it (short launches would otherwise count
            # the ~20 us of Python per call)
            park_gpu(0.08)
            vc.pipeline_device(hub, net_g, 0, audio_dev, 0, "v2", 0.33, index, args.index_rate, args.f0)
        n, ms, flops = probe.summary(engine=1)  # dominant family: the split-operand conv engine
        n32, ms32, fl32 = probe.summary(engine=0)
        n64, ms64, fl64 = probe.summary(engine=2)
        groups, peak = probe.by_passes()
        timing = "HIP events around each launch (bench.py ConvProbe)"
        # the same pass again under torch.profiler, whose kernel records are the device's own start / end stamps
        # (what rocprofv3's kernel trace reads): the events above add a few us of their own to every launch
        fam_ms = {}
        prof = profiler_kernel_times(lambda: vc.pipeline_device(hub, net_g, 0, audio_dev, 0, "v2", 0.33, index,
                                                                args.index_rate, args.f0), fam_ms)
        if prof and sum(v[0] for v in prof.values()) == n:
            ev_ms = {p: g[1] for p, g in groups.items()}
            for p, g in groups.items():
                if p in prof:
                    g[1] = prof[p][1]
            if all(p in prof for p in groups):
                ms = sum(g[1] for g in groups.values())
                timing = ("device kernel stamps (torch.profiler over a second pass; HIP-event time of the "
                          f"instrumented pass {sum(ev_ms.values()):.3f} ms)")
            else:
                for p in groups:
                    groups[p][1] = ev_ms[p]
        achieved = flops / (ms * 1e-3) / 1e12
        traffic, tsrc = (pmc_traffic("x6") if (args.sr, args.f0, args.precision, args.index_rate, args.seconds)
                         == (48000, "rmvpe", "fp32", 0.0, 30.0) else (None, None))
        alg_bytes = probe.algorithmic_bytes(engine=1)
        names = {1: "bf16 x1", 3: "split-bf16 x3", 6: "split-bf16 x6", 7: "split-bf16 x6 split-acc", 16: "split-fp16 x3"}
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 2), "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4),
                # HBM bytes per launch of the family from PMC (default 48k / rmvpe / fp32 step only), beside the
                # algorithmic bytes per launch measured here
                "traffic": traffic,
                "traffic_unit": (f"bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/{tsrc})" if traffic
                                 else f"null: {tsrc}"),
                "algorithmic_bytes_per_launch": round(alg_bytes),
                "traffic_over_algorithmic": round(traffic / alg_bytes, 3) if traffic else None,
                "kernel": "conv_x6_kernel<*> + resblock_x6_kernel<*> (implicit-GEMM convs / fused ResBlock conv "
                          "pairs on the split-operand MFMA engine); achieved = algorithmic FLOPs / kernel time; peak = "
                          "the FLOP-weighted ceiling of the pass sets that ran: sum FLOPs / sum (FLOPs / (2.5 PF dense "
                          "16-bit MFMA / passes per product))",
                "by_pass_set": {names.get(p, str(p)): {"launches": g[0], "kernel_ms": round(g[1], 3),
                                                       "gflop": round(g[2] / 1e9, 1),
                                                       "tflops": round(g[2] / max(g[1], 1e-9) / 1e9, 2),
                                                       "peak": round(pass_peak(p), 1)}
                                for p, g in sorted(groups.items())},
                "launches_per_step": n, "avg_launch_ms": round(ms / max(n, 1), 4), "timing": timing,
                "algorithmic_gflop_per_step": round(flops / 1e9, 1), "kernel_ms_per_step": round(ms, 3),
                "f32_engine": {"launches": n32, "kernel_ms": round(ms32, 3), "gflop": round(fl32 / 1e9, 1),
                               "tflops": round(fl32 / max(ms32, 1e-9) / 1e9, 2), "peak": PEAK_F32_MFMA_TFLOPS},
                "f64_engine": {"launches": n64, "kernel_ms": round(ms64, 3), "gflop": round(fl64 / 1e9, 1),
                               "tflops": round(fl64 / max(ms64, 1e-9) / 1e9, 2), "peak": PEAK_F64_MFMA_TFLOPS,
                               "measured_ceiling": F64_MEASURED_TFLOPS,
                               "note": "the f64 RMVPE's convs (rmvpe64.hip: conv64_kernel with its split-K reduce, and "
                                       "the Winograd F(4x4,3x3) convs at their direct-conv algorithmic FLOPs); peak = "
                                       "the f64 matrix spec, measured_ceiling = what the chip sustains in f64 on real "
                                       "operands (power-bound, DESIGN.md §4 conv64)"},
                # the other kernel families of the same per-call pass, device kernel stamps (torch.profiler)
                "families": family_rooflines(probe.aux, fam_ms) if fam_ms else None}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline()
    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 3), "unit": "audio-s/s", "n_gpus": world,
                "value_per_gpu": round(value / world, 3), "world_size": world, "devices_used": min(world, ndev),
                "collective": ("none" if world == 1 else
                               "RCCL gather over xGMI" if backend == "nccl" else "gloo (ranks share a GPU)"),
                "waveforms_gathered_per_step": gathered_per_step,
                "output": ("host-visible: each clip's waveform copied to pinned host memory inside the timed region "
                           "(the reference signature's .cpu(), SURVEY §8(d))" if host_visible else
                           "HBM-resident (gathered to rank 0's device)" if mine is not None else
                           "HBM-resident (--hbm-output)"),
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "strong" if mine is not None else "weak", "vs_baseline": None,
                "dtype": DTYPES[args.precision],
                "data": "synthetic 16 kHz audio (SURVEY §8d generator), random-init weights of the true shapes",
                "config": {"workload": (f"BASELINE configs[3]: {args.utterances} x {args.seconds:g} s utterances "
                                        f"({args.utterances * args.seconds / 3600:g} h) sharded longest-first over "
                                        f"{world} GPU(s), one clip stream per rank, waveforms gathered to rank 0 by "
                                        f"grouped send/recv; VC.pipeline {args.sr // 1000}k v2, ContentVec-768, "
                                        f"{args.f0} f0, " if mine is not None else
                                        f"VC.pipeline {args.sr // 1000}k v2, ContentVec-768, {args.f0} f0, "
                                        f"{'one' if len(clips) == 1 else f'{len(clips)} x'} "
                                        f"{args.seconds:g} s clip per GPU per step, ")
                                       + (f"IVF-Flat index_rate {args.index_rate:g}" if index is not None else "no index")
                                       + ", protect 0.33" + (", hipGraph replay per clip" if args.graph else "")
                                       + (", clip stream (clip k+1 f0/features under clip k synthesizer)"
                                          if args.stream else "")
                                       + (f", RMVPE + ContentVec batched {args.batch} clips per pass"
                                          if args.batch > 1 else ""),
                           "model": f"RVC v2 {args.sr // 1000}k (NSF-HiFiGAN) + ContentVec + {args.f0}",
                           "global_batch": args.utterances if mine is not None else world * len(clips),
                           "seq_len": int(args.seconds * 16000), "parallelism": f"utterance-sharded x{world}",
                           "output_seconds_per_clip": round(audio_s, 4)},
                "per_call": per_call, "roofline": roof, "cpu_baseline": cpu}
        if mine is not None:
            line["utterances_per_rank"] = len(mine)
            line["gather_bytes_recv_per_step"] = p2p.get("bytes_recv", 0)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def launch_ranks(n):
    """``bench.py --gpus N`` without a launcher: run ``torch.distributed.run --nproc-per-node N`` over this
    same script as a child process (rendezvous on 127.0.0.1) and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


if __name__ == "__main__":
    sys.exit(main())
