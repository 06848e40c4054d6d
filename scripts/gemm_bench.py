"""A/B of the conv engine on ContentVec's pointwise (K = 1) GEMM shapes at one 30 s clip (1599 frames):
pass set x split-K target, HIP events, max relative error against an f64 product.

    python scripts/gemm_bench.py [--reps 20]
"""
import argparse
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))

SHAPES = [(3072, 768, 1599), (768, 3072, 1599), (2304, 768, 1599), (768, 768, 1599)]  # Co, Ci, N


def run(prec, reps, only=""):
    import torch
    from rvc_amd import ops
    ops.set_precision(prec)
    g = torch.Generator().manual_seed(0)
    tot = 0.0
    for i, (Co, Ci, N) in enumerate(SHAPES):
        if only and str(i) not in only.split(","):
            continue
        w = torch.randn(Co, Ci, 1, generator=g) / Ci ** 0.5
        b = torch.randn(Co, generator=g)
        conv = ops.Conv(w, b, device="cuda")
        x = torch.randn(Ci, N, generator=g).cuda()
        y = torch.empty(Co, N, device="cuda")
        fn = lambda: conv(x, out=y)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        tot += us
        ref = (w[:, :, 0].double() @ x.cpu().double()) + b.double()[:, None]
        err = float(((y.cpu().double() - ref).abs().max() / ref.abs().max()))
        print(f"  {prec:7s} {Co:5d}x{Ci:5d}x{N}: "
              f"{us:7.1f} us  {2 * Co * Ci * N / us / 1e6:6.1f} TF/s  max rel err {err:.2e}", flush=True)
    print(f"  total {tot:.1f} us", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--child", default="")
    ap.add_argument("--precisions", default="fp32,f16x3")
    ap.add_argument("--only", default="", help="comma list of shape indices")
    ap.add_argument("--envs", default="RVC_SPLITK_TILES=512;RVC_SPLITK_TILES=256;RVC_SPLITK_TILES=0",
                    help="';'-separated environment settings, each a ','-separated list of NAME=VALUE")
    args = ap.parse_args()
    if args.child:
        return run(args.child, args.reps, args.only)
    for setting in args.envs.split(";"):
        env = dict(os.environ, **dict(kv.split("=", 1) for kv in setting.split(",") if kv))
        for prec in args.precisions.split(","):
            print(f"[{setting}]", flush=True)
            rc = subprocess.call([sys.executable, __file__, "--child", prec, "--reps", str(args.reps), "--only",
                                  args.only], env=env)
            if rc:
                return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
