"""Conv-engine A/B bench on the generator's dominant shapes (HIP events; lrelu pre-activation and
residual epilogue as in the ResBlocks).  Select a library build with RVC_AMD_LIB.

    RVC_AMD_LIB=path/to/librvc_amd.so python scripts/conv_bench.py [--reps 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))

import torch  # noqa: E402

SHAPES = [  # C, K, dil, L
    (256, 3, 1, 38376), (256, 11, 1, 38376),
    (128, 3, 1, 383760), (128, 7, 3, 383760), (128, 11, 5, 383760),
    (64, 3, 1, 767520), (64, 11, 1, 767520),
    (32, 3, 1, 1535040), (32, 11, 1, 1535040),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", type=str, default="", help="comma list of shape indices")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--check", action="store_true", help="compare each shape with the f32-MFMA engine")
    ap.add_argument("--amax", action="store_true", help="hand each conv its input's |max| cell (the generator's "
                                                        "amax side channel: split-fp16 without the tile pre-pass)")
    args = ap.parse_args()
    from rvc_amd import ops
    ops.set_precision(args.precision)
    print("lib:", ops._lib.LIB_PATH)
    g = torch.Generator().manual_seed(0)
    tot_ms = tot_fl = 0.0
    shapes = [SHAPES[int(i)] for i in args.only.split(",")] if args.only else SHAPES
    for C, K, d, L in shapes:
        w = torch.randn(C, C, K, generator=g) / (C * K) ** 0.5
        conv = ops.Conv(w, torch.randn(C, generator=g), device="cuda")
        x = torch.randn(C, L, generator=g).cuda()
        res = torch.randn(C, L, generator=g).cuda()
        y = torch.empty(C, L, device="cuda")
        p = d * (K - 1) // 2
        akw = {}
        if args.amax:
            import numpy as np
            cell = ops.AmaxSlots(1, "cuda")
            cell.words[0] = int(np.float32(x.abs().max().item()).view(np.int32))
            akw["amax_in"] = cell[0]
        fn = lambda: conv(x, pad=p, dil=d, out=y, res=res, in_act=ops.ACT_LRELU, in_slope=0.1, **akw)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        fl = 2.0 * C * C * K * L
        tot_ms += ms
        tot_fl += fl
        chk = ""
        if args.check:
            wx, conv.wx = conv.wx, None  # f32-MFMA engine
            yr = torch.empty_like(y)
            conv(x, pad=p, dil=d, out=yr, res=res, in_act=ops.ACT_LRELU, in_slope=0.1)
            conv.wx = wx
            fn()
            torch.cuda.synchronize()
            rel = float((y - yr).pow(2).mean().sqrt() / (yr - res).pow(2).mean().sqrt())
            chk = f"  rel err vs f32 engine {rel:.2e}"
            assert rel < {"fp32": 1e-5, "fp32x6": 1e-5, "f16x3": 1e-5, "bf16x3": 1e-4, "bf16": 2e-2}[args.precision], chk
        print(f"C={C:4d} K={K:2d} d={d} L={L:8d}: {ms * 1e3:9.1f} us {fl / ms / 1e9:7.1f} TFLOP/s{chk}")
    print(f"total {tot_ms:.3f} ms, {tot_fl / tot_ms / 1e9:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
