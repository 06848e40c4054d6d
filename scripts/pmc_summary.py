"""Summarise rocprofv3 --pmc csv passes: per kernel-name pattern, mean counter value per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

pat = sys.argv[2] if len(sys.argv) > 2 else "conv_x6"
for d in sys.argv[1].split(","):
    acc = defaultdict(list)
    for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (disp, name), v in per.items():
            acc[name].append(v)
    print(d, {k: f"{sum(v) / len(v):.4g}" for k, v in sorted(acc.items())})
