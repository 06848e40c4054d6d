"""Group a rocprofv3 kernel_trace.csv by (kernel, grid): total ms per pass, calls per pass, mean us per call.

    python scripts/ktrace_group.py gpurun_out/x/run_kernel_trace.csv PASSES [name-filter]
"""
import csv
import re
import sys
from collections import defaultdict

path, passes = sys.argv[1], float(sys.argv[2])
flt = sys.argv[3] if len(sys.argv) > 3 else ""
acc = defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if flt not in name:
        continue
    grid = tuple(int(r.get(f"Grid_Size_{a}", r.get(f"Grid_{a}", 0)) or 0) for a in "XYZ")
    wg = tuple(int(r.get(f"Workgroup_Size_{a}", 0) or 0) for a in "XYZ")
    blocks = tuple(g // max(w, 1) for g, w in zip(grid, wg))
    acc[(re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0][:70], blocks)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
tot = sum(sum(v) for v in acc.values())
print(f"total {tot / passes / 1e3:.2f} ms per pass")
for (name, blocks), v in rows[:40]:
    print(f"{sum(v) / passes / 1e3:7.3f} ms {len(v) / passes:6.1f} x {sum(v) / len(v):8.1f} us  {blocks}  {name}")
