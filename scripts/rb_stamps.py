"""Where a fused ResBlock pair's tile spends its cycles (resblock_x6_kernel, csrc/resblock.hip): the in-kernel s_memtime
stamps of the diagnostic build (-DRVC_CONV_STAMPS=1 -> rvc-maker_amd/lib/s/librvc_amd.so), per tile phase of compute
wave 0 -- S0 wait, c1 k-steps, c1 epilogue up to B_T (the T tile's |max| agreement, split-fp16), T write + S1, c2
k-steps, c2 epilogue -- and of the first loader wave (tile k+1's loads issued, staged), against the MFMA-bound cycles
of each conv (per SIMD: 2 compute waves x NCH * K k-steps x FM * FN * NP MFMAs x 16 cycles).

    RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so python scripts/rb_stamps.py [--out f.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

W, NT = 256, 31  # RB_STAMP_W, RB_STAMP_NT
# the generator's fused pairs at 48k, 30 s (synth.py: stages 2 and 3), and the dilations each kernel size takes
SHAPES = [("c64_k3_d1", 64, 3, 1, 767520), ("c64_k7_d3", 64, 7, 3, 767520), ("c64_k11_d5", 64, 11, 5, 767520),
          ("c32_k3_d1", 32, 3, 1, 1535040), ("c32_k7_d3", 32, 7, 3, 1535040), ("c32_k11_d5", 32, 11, 5, 1535040)]


def analyse(st, C, K, passes, wide):
    ok = st[:, 248] > 0
    st = st[ok].astype(np.float64)
    nt = int(np.median(st[:, 251]))
    nt_s = min(nt, NT)
    ph = {k: [] for k in ("s0_wait", "c1", "c1_epi_to_BT", "T_write_S1", "c2", "c2_epi", "loader_load_issue",
                          "loader_stage", "tile")}
    for k in range(1, nt_s - 1):  # steady tiles (the first and last have the prologue / drain)
        b = 8 * k
        prev_epi = st[:, 8 * (k - 1) + 5]
        ph["s0_wait"].append(st[:, b] - prev_epi)
        ph["c1"].append(st[:, b + 1] - st[:, b])
        ph["c1_epi_to_BT"].append(st[:, b + 2] - st[:, b + 1] if np.any(st[:, b + 2]) else st[:, b + 3] * 0)
        ph["T_write_S1"].append(st[:, b + 3] - (st[:, b + 2] if np.any(st[:, b + 2]) else st[:, b + 1]))
        ph["c2"].append(st[:, b + 4] - st[:, b + 3])
        ph["c2_epi"].append(st[:, b + 5] - st[:, b + 4])
        ph["loader_load_issue"].append(st[:, b + 6] - st[:, b])
        ph["loader_stage"].append(st[:, b + 7] - st[:, b + 6])
        ph["tile"].append(st[:, 8 * (k + 1)] - st[:, b])
    med = {k: float(np.median(np.concatenate(v))) for k, v in ph.items() if v}
    nch = C // 32
    f16 = passes == 16
    np_ = 3 if passes in (3, 16) else passes
    fm, fn = (2 if C == 128 or (C == 64 and wide) else 1), 4  # RbGeom: row fragments per wave (WIDE at C = 64)
    rg = C // 16 // fm
    med["outputs_per_tile"] = 16 * (4 * (8 // rg) - 1)
    mfma = 2 * nch * K * fm * fn * np_ * 16  # per SIMD per conv: 2 compute waves per SIMD
    med["mfma_bound_per_conv"] = mfma
    med["mfma_busy_tile"] = 2 * mfma / max(med["tile"], 1)
    med["tiles_per_block"] = nt
    med["block_cycles"] = float(np.median(st[:, 253] - st[:, 248]))
    return med


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--wide64", type=int, default=1, help="the C = 64 geometry (rvc_resblock_set_wide64)")
    args = ap.parse_args()
    from rvc_amd import _lib, ops
    from rvc_amd.ops import Conv
    lib = _lib.load()
    ops.set_precision(args.precision)
    nb = 1024
    buf = torch.zeros(nb * W, dtype=torch.int64, device="cuda")
    import ctypes
    if lib.rvc_resblock_set_stamps(ctypes.c_void_p(buf.data_ptr()), buf.numel() * 8) != 0:
        raise SystemExit("this library has no stamps: build with EXTRA=-DRVC_CONV_STAMPS=1")
    lib.rvc_resblock_set_wide64(args.wide64)
    print("lib:", _lib.LIB_PATH, "precision:", args.precision, "wide64:", args.wide64)
    g = torch.Generator().manual_seed(0)
    out = {}
    from torch.profiler import ProfilerActivity, profile
    for name, C, K, d, L in SHAPES:
        x = torch.randn(C, L, generator=g).to("cuda")
        y = torch.empty_like(x)
        c1 = Conv(torch.randn(C, C, K, generator=g) * 0.05, torch.randn(C, generator=g) * 0.1, device="cuda")
        c2 = Conv(torch.randn(C, C, K, generator=g) * 0.05, torch.randn(C, generator=g) * 0.1, device="cuda")
        for _ in range(3):
            ops.resblock_pair(x, y, c1, c2, d, 0.1)
        torch.cuda.synchronize()
        buf.zero_()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            ops.resblock_pair(x, y, c1, c2, d, 0.1)
            torch.cuda.synchronize()
        kn = [e for e in prof.events() if "resblock_x6_kernel" in e.name]
        us = kn[0].time_range.elapsed_us() if kn else float("nan")
        st = buf.view(nb, W).cpu().numpy().astype(np.uint64)
        r = analyse(st, C, K, ops.rb_passes(K), args.wide64 and ops.rb_passes(K) != 6)
        r.update(kernel_us=us, tflops=4.0 * C * C * K * L / us / 1e6, passes=ops.rb_passes(K))
        out[name] = r
        print(f"{name:11s} {us:7.1f} us {r['tflops']:6.1f} TF  tiles/block {r['tiles_per_block']} x {r['outputs_per_tile']}"
              f"  tile {r['tile']:.0f} cyc "
              f"(MFMA-bound {2 * r['mfma_bound_per_conv']}, busy {r['mfma_busy_tile']:.2f}):  S0 wait {r['s0_wait']:.0f}"
              f" | c1 {r['c1']:.0f} | c1 epi->B_T {r['c1_epi_to_BT']:.0f} | T + S1 {r['T_write_S1']:.0f} | c2 {r['c2']:.0f}"
              f" | c2 epi {r['c2_epi']:.0f};  loader: loads issued +{r['loader_load_issue']:.0f}, staged "
              f"{r['loader_stage']:.0f}")
    lib.rvc_resblock_set_stamps(None, 0)
    lib.rvc_resblock_set_wide64(-1)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
