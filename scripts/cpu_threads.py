"""CPU baseline thread scaling on the GPU box's host: the torch-CPU oracle (bench.cpu_baseline) on a 10 s clip at
several torch thread counts, to choose and state bench.py's cpu_baseline thread count.

    python scripts/cpu_threads.py 8 16 32 64
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    counts = [int(a) for a in sys.argv[1:]] or [8, 16, 32, 64]
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    rows = []
    for n in counts:
        torch.set_num_threads(n)
        t0 = time.perf_counter()
        r = bench.cpu_baseline(seconds=10.0)
        rows.append({"threads": n, "xRT": r["value"], "wall_s": round(time.perf_counter() - t0, 2)})
        print(json.dumps(rows[-1]), flush=True)
    best = max(rows, key=lambda r: r["xRT"])["threads"]
    print(json.dumps({"os_cpu_count": os.cpu_count(), "affinity": aff, "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
                      "rows": rows, "best_threads": best}))


if __name__ == "__main__":
    main()
