"""Compare rocprofv3 kernel_stats.csv files: total ms per kernel name (normalised per pipeline pass)."""
import csv
import sys

files = sys.argv[1:]
tabs = []
for f in files:
    path, _, div = f.partition(":")
    d = {}
    for r in csv.DictReader(open(path)):
        d[r["Name"][:90]] = (float(r["TotalDurationNs"]) / 1e6 / float(div or 1), int(r["Calls"]) / float(div or 1))
    tabs.append(d)
names = sorted(set().union(*tabs), key=lambda n: -max(t.get(n, (0, 0))[0] for t in tabs))
for n in names[:30]:
    print(" | ".join(f"{t.get(n, (0, 0))[0]:7.2f} ms {t.get(n, (0, 0))[1]:6.1f}" for t in tabs), " ", n)
print(" | ".join(f"{sum(v[0] for v in t.values()):7.2f} ms total" for t in tabs))
