"""Is a VC.pipeline_device step host-bound?  Times the host issue of one step (return of the call,
no sync) against the step's completion (after sync).

    python scripts/host_overhead.py [--seconds 30]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=30.0)
    args = ap.parse_args()
    from rvc_amd import synthetic
    vc, hub, net_g = bench.build_models("cuda:0")
    audio = torch.from_numpy(synthetic.synthetic_audio(args.seconds, seed=1000)).cuda()
    for _ in range(2):
        vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33)
    torch.cuda.synchronize()
    for _ in range(3):
        t0 = time.perf_counter()
        vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"host issue {1e3 * (t1 - t0):8.2f} ms   step complete {1e3 * (t2 - t0):8.2f} ms")


if __name__ == "__main__":
    main()
