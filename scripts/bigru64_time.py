"""Times the library's f64 BiGRU recurrence (ops.bigru64_batched) at the 30 s clip's length (HIP events).
    python scripts/bigru64_time.py [--T 3232] [--B 1]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=3232)
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--save", default="", help="write y (f64, .npy) for an offline comparison")
    args = ap.parse_args()
    from rvc_amd import ops
    dev, B, T = "cuda", args.B, args.T
    g = torch.Generator().manual_seed(0)
    gi = (torch.randn(B, 1536, T, generator=g, dtype=torch.float64) * 0.5).to(dev)
    whh = (torch.randn(2, 768, 256, generator=g, dtype=torch.float64) * 0.06).to(dev)
    bhh = (torch.randn(2, 768, generator=g, dtype=torch.float64) * 0.1).to(dev)
    y = torch.empty(B, 512, T, device=dev, dtype=torch.float64)
    gran = torch.zeros(ops.GRU64_GRAN * min(B, ops.GRU_B_MAX), dtype=torch.int64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.bigru64_batched(gi, whh, bhh, y, gran, err, B, T)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        ops.bigru64_batched(gi, whh, bhh, y, gran, err, B, T)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    print(f"bigru64 B={B} T={T}: {ms:.3f} ms ({ms * 1e3 / T:.3f} us/step) "
          f"err={int(err.item())} checksum={float(y.double().sum()):.12e}")
    if args.save:
        import numpy as np
        np.save(args.save, y.cpu().numpy())


if __name__ == "__main__":
    main()
