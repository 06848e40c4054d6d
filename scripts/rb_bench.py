"""Fused ResBlock pair timings at the generator's 48k shapes (HIP events):
    python scripts/rb_bench.py [--reps 5]      (RVC_AMD_LIB selects a variant build)"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--c128", action="store_true", help="the 128-channel pair (stage 1, 30 s 48k): fused vs two launches")
    args = ap.parse_args()
    if args.c128:
        return c128(args)
    from rvc_amd import ops
    from rvc_amd.ops import Conv
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    tot_ms = tot_fl = 0.0
    with ops.precision(args.precision):
        for C, L in ((64, 767520), (32, 1535040)):
            x = torch.randn(C, L, generator=g).to(dev)
            y = torch.empty_like(x)
            for K in (3, 7, 11):
                c1 = Conv(torch.randn(C, C, K, generator=g) * 0.05, torch.randn(C, generator=g) * 0.1, device=dev)
                c2 = Conv(torch.randn(C, C, K, generator=g) * 0.05, torch.randn(C, generator=g) * 0.1, device=dev)
                for d, acc in ((1, False), (5, True)):
                    ops.resblock_pair(x, y, c1, c2, d, 0.1, accumulate=acc)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.reps):
                        ops.resblock_pair(x, y, c1, c2, d, 0.1, accumulate=acc)
                    e1.record()
                    torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1) / args.reps
                    fl = 4.0 * C * C * K * L
                    tot_ms += ms * 3
                    tot_fl += fl * 3
                    print(f"C={C:3d} K={K:2d} d={d} acc={int(acc)}: {ms * 1e3:7.1f} us  {fl / ms / 1e9:6.1f} TF/s")
    print(f"total (x3 per shape): {tot_ms:.2f} ms, {tot_fl / tot_ms / 1e9:.1f} TF/s")


def c128(args):
    from rvc_amd import ops
    from rvc_amd.ops import ACT_LRELU, Conv
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    C, L = 128, 383760
    x = torch.randn(C, L, generator=g).to(dev)
    y = torch.empty_like(x)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps * 1e3

    with ops.precision(args.precision):
        for K in (3, 7, 11):
            c1 = Conv(torch.randn(C, C, K, generator=g) * 0.03, torch.randn(C, generator=g) * 0.1, device=dev)
            c2 = Conv(torch.randn(C, C, K, generator=g) * 0.03, torch.randn(C, generator=g) * 0.1, device=dev)
            for d in (1, 5):
                def two():
                    t1 = c1(x, pad=(K * d - d) // 2, dil=d, in_act=ACT_LRELU, in_slope=0.1)
                    c2(t1, pad=(K - 1) // 2, out=y, res=x, in_act=ACT_LRELU, in_slope=0.1)
                us2 = timed(two)
                try:
                    usf = timed(lambda: ops.resblock_pair(x, y, c1, c2, d, 0.1))
                except RuntimeError:
                    usf = float("nan")
                print(f"C=128 K={K:2d} d={d} passes={ops.rb_passes(K)}: two launches {us2:7.1f} us, fused {usf:7.1f} us")


if __name__ == "__main__":
    main()
