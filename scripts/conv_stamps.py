"""Where a split-operand conv block spends its cycles: the x6 engine's in-kernel s_memtime stamps (diagnostic build,
-DRVC_CONV_STAMPS=1 -> rvc-maker_amd/lib/s/librvc_amd.so) per phase -- prologue (weight prefetch issue, split-fp16
tile-|max| pre-pass, chunk 0 staging), each chunk's compute segment and barrier wait (compute wave 0) against the
loaders' staging and wait (first loader wave), epilogue -- against the MFMA-bound cycles of a chunk, plus the CU
timeline (blocks per CU, gaps between a CU's consecutive blocks).

    RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so python scripts/conv_stamps.py [--precision fp32|f16x3|...] [--only i,j]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

W = 256  # X6_STAMP_W
SHAPES = [  # name, Ci, Co, K, dil, L, pre-activation (ResBlock convs: lrelu + residual; GEMMs: none)
    ("rb128_k11", 128, 128, 11, 5, 383760, True),
    ("rb128_k11_nores", 128, 128, 11, 5, 383760, None),
    ("rb128_k11_256blk", 128, 128, 11, 5, 256 * 256, True),  # one block per CU: the epilogue against HBM contention
    ("rb128_k11_32blk", 128, 128, 11, 5, 32 * 256, True),
    ("rb128_k11_128blk", 128, 128, 11, 5, 128 * 256, True),
    ("rb128_k11_192blk", 128, 128, 11, 5, 192 * 256, True),
    ("rb128_k7", 128, 128, 7, 3, 383760, True),
    ("rb128_k3", 128, 128, 3, 1, 383760, True),
    ("rb256_k3", 256, 256, 3, 1, 95940, True),
    ("rb256_k11", 256, 256, 11, 1, 95940, True),
    ("cv_fc1", 768, 3072, 1, 1, 1599, False),
    ("cv_fc2", 3072, 768, 1, 1, 1599, False),
    ("cv_qkv", 768, 2304, 1, 1, 1599, False),
    ("te_ffn", 192, 768, 3, 1, 3200, False),
]


def mfma_cycles_per_chunk(name, K):
    """MFMA-pipe cycles one SIMD needs per 32-channel chunk: its compute waves x K k-steps x MFMAs per k-step x 16."""
    args = [int(a) if a.isdigit() else a for a in name.split("<", 1)[1].split(">")[0].replace(" ", "").split(",")]
    FM, FN, WM, WN, _, NP = args[:6]
    waves_per_simd = WM * WN / 4
    return waves_per_simd * K * FM * FN * NP * 16


def analyse(st, nblk, K, kname):
    st = st[:nblk]
    ok = st[:, 0] > 0
    st = st[ok]
    nch = st[:, 12].astype(np.int64)
    res = {"blocks": int(len(st)), "chunks_per_block": int(np.median(nch))}
    d = lambda a, b: (st[:, b].astype(np.float64) - st[:, a].astype(np.float64))  # noqa: E731
    res["block_cycles_med"] = float(np.median(d(0, 7)))
    res["prologue_compute_med"] = float(np.median(d(0, 5)))  # start -> chunk 0 ready
    if np.any(st[:, 4]):
        res["f16_scale_wait_med"] = float(np.median(d(3, 4)))
        res["loader_prepass_med"] = float(np.median(d(8, 9)))
    res["loader_chunk0_med"] = float(np.median(d(9 if np.any(st[:, 9]) else 8, 10)))
    res["loop_med"] = float(np.median(d(5, 6)))
    res["epilogue_med"] = float(np.median(d(6, 7)))
    if np.any(st[:, 14]):
        res["epilogue_issue_med"] = float(np.median(d(6, 14)))
    nc = min(int(np.median(nch)), 60)
    comp, cwait, lbusy, lwait = [], [], [], []
    for c in range(nc):
        a, r = 16 + 4 * c, 16 + 4 * c + 1
        prev_rel = st[:, 5] if c == 0 else st[:, 16 + 4 * (c - 1) + 1]
        comp.append(np.median(st[:, a].astype(np.float64) - prev_rel))
        cwait.append(np.median(st[:, r].astype(np.float64) - st[:, a]))
        la, lr = 16 + 4 * c + 2, 16 + 4 * c + 3
        lprev = st[:, 10] if c == 0 else st[:, 16 + 4 * (c - 1) + 3]
        lbusy.append(np.median(st[:, la].astype(np.float64) - lprev))
        lwait.append(np.median(st[:, lr].astype(np.float64) - st[:, la]))
    mf = mfma_cycles_per_chunk(kname, K)
    res["per_chunk"] = {"compute_med": float(np.median(comp)), "barrier_wait_med": float(np.median(cwait)),
                        "loader_busy_med": float(np.median(lbusy)), "loader_wait_med": float(np.median(lwait)),
                        "mfma_bound": mf}
    res["mfma_busy_in_loop"] = float(mf * nc / max(res["loop_med"], 1))
    res["mfma_busy_block"] = float(mf * nc / max(res["block_cycles_med"], 1))
    # CU timeline: HW_ID (CU / SE fields) + XCC, blocks per CU, gap between a CU's consecutive blocks (realtime, 10 ns)
    hw = st[:, 2].astype(np.int64)
    cu_key = (st[:, 13].astype(np.int64) << 32) | ((hw >> 8) & 0xFF)  # XCC, then HW_ID's CU / SH / SE fields
    rt = st[:, 1].astype(np.float64)
    dur_rt = (d(0, 7) / max(res["block_cycles_med"], 1)) * 0  # placeholder (memtime and realtime differ in rate)
    gaps, per_cu, ends = [], [], []
    clk = None
    for k in np.unique(cu_key):
        idx = np.where(cu_key == k)[0]
        order = idx[np.argsort(rt[idx])]
        per_cu.append(len(order))
        for a, b in zip(order[:-1], order[1:]):
            gaps.append(rt[b] - rt[a])
            # the next block's start against this block's end, in the CU's own shader clock
            ends.append(float(st[b, 0]) - float(st[a, 7]) if st[b, 0] > st[a, 7] else np.nan)
    res["cus_seen"] = int(len(per_cu))
    res["blocks_per_cu_med"] = float(np.median(per_cu))
    if gaps:
        res["cu_block_period_us_med"] = float(np.median(gaps)) / 100.0  # 100 MHz realtime
    res["launch_span_us"] = float((rt.max() - rt.min()) / 100.0)
    if ends:
        e = np.array(ends, dtype=np.float64)
        res["next_block_start_after_end_cyc_med"] = float(np.nanmedian(e)) if np.isfinite(e).any() else None
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default="")
    ap.add_argument("--amax", action="store_true", help="hand each conv its input's |max| (the amax side channel, "
                                                        "as the generator does): no split-fp16 pre-pass")
    args = ap.parse_args()
    from rvc_amd import _lib, ops
    lib = _lib.load()
    ops.set_precision(args.precision)
    print("lib:", _lib.LIB_PATH, "precision:", args.precision)
    nb_max = 32768
    buf = torch.zeros(nb_max * W, dtype=torch.int64, device="cuda")
    if lib.rvc_conv1d_set_stamps(ctypes_ptr(buf), buf.numel() * 8) != 0:
        raise SystemExit("this library has no stamps: build with EXTRA=-DRVC_CONV_STAMPS=1")
    g = torch.Generator().manual_seed(0)
    shapes = [SHAPES[int(i)] for i in args.only.split(",")] if args.only else SHAPES
    out = {}
    from torch.profiler import ProfilerActivity, profile
    for name, Ci, Co, K, d, L, rb in shapes:
        w = torch.randn(Co, Ci, K, generator=g) / (Ci * K) ** 0.5
        conv = ops.Conv(w, torch.randn(Co, generator=g), device="cuda")
        x = torch.randn(Ci, L, generator=g).cuda()
        res = torch.randn(Co, L, generator=g).cuda() if rb else None  # rb None: the ResBlock conv minus its residual
        y = torch.empty(Co, L, device="cuda")
        p = d * (K - 1) // 2
        kw = dict(pad=p, dil=d, out=y, res=res)
        if args.amax:
            cell = ops.AmaxSlots(1, "cuda")
            cell.words[0] = int(np.float32(x.abs().max().item()).view(np.int32))
            kw["amax_in"] = cell[0]
        if rb is not False:
            kw.update(in_act=ops.ACT_LRELU, in_slope=0.1)
        for _ in range(3):
            conv(x, **kw)
        torch.cuda.synchronize()
        buf.zero_()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            conv(x, **kw)
            torch.cuda.synchronize()
        kn = [e for e in prof.events() if "conv_x6_kernel" in e.name]
        if not kn:
            print(f"{name}: no x6 launch (engine {ops.LAST_CONV_ENGINE})")
            continue
        kname = kn[0].name.replace("(anonymous namespace)::", "").replace("void ", "")
        us = kn[0].time_range.elapsed_us()
        st = buf.view(nb_max, W).cpu().numpy().astype(np.uint64)
        nblk = int((st[:, 0] > 0).sum())
        r = analyse(st, nb_max, K, kname)
        r.update(kernel=kname, kernel_us=us, passes=ops.LAST_CONV_PASSES, tflops=2.0 * Ci * Co * K * L / us / 1e6)
        # effective clock: block cycles vs block realtime is not stamped; infer from the launch: cycles per us
        out[name] = r
        pc = r["per_chunk"]
        print(f"{name:10s} {kname[:48]:48s} {us:8.1f} us {r['tflops']:6.1f} TF  blocks {r['blocks']} "
              f"({r['blocks_per_cu_med']:.0f}/CU, period {r.get('cu_block_period_us_med', 0):.1f} us) chunks {r['chunks_per_block']}")
        print(f"   block {r['block_cycles_med']:.0f} cyc = prologue {r['prologue_compute_med']:.0f}"
              + (f" (f16 scale wait {r['f16_scale_wait_med']:.0f}, loader pre-pass {r['loader_prepass_med']:.0f})"
                 if 'f16_scale_wait_med' in r else "")
              + f" + loop {r['loop_med']:.0f} + epilogue {r['epilogue_med']:.0f} (issued after {r.get('epilogue_issue_med', 0):.0f});  loader chunk0 {r['loader_chunk0_med']:.0f}")
        print(f"   CU period {r.get('cu_block_period_us_med', 0):.1f} us; next block starts "
              f"{r.get('next_block_start_after_end_cyc_med')} cyc after wave 0's epilogue stamp")
        print(f"   per chunk: compute {pc['compute_med']:.0f} + barrier wait {pc['barrier_wait_med']:.0f} (MFMA-bound "
              f"{pc['mfma_bound']:.0f}); loader busy {pc['loader_busy_med']:.0f} wait {pc['loader_wait_med']:.0f};  "
              f"MFMA busy in loop {r['mfma_busy_in_loop']:.2f}, over the block {r['mfma_busy_block']:.2f}")
    lib.rvc_conv1d_set_stamps(None, 0)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


def ctypes_ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


if __name__ == "__main__":
    main()
