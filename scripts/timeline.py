"""Stream timeline from a rocprofv3 kernel_trace.csv: per queue/stream busy time (union of kernel intervals),
gaps, and the kernels that fill them, over the window of the last N clips of a clip-stream bench run.

    python scripts/timeline.py TRACE.csv [--from-kernel NAME] [--top 15]
"""
import argparse
import collections
import csv


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0][:70]


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--top", type=int, default=15)
ap.add_argument("--clips", type=int, default=4, help="window = the last N clips (between peak-normalise ends)")
ap.add_argument("--marker", default="absmax_kernel", help="the kernel that ends a clip")
a = ap.parse_args()
import gzip
rows = list(csv.DictReader(gzip.open(a.trace, "rt") if a.trace.endswith(".gz") else open(a.trace)))
key_q = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key_q], r["Kernel_Name"]) for r in rows]
ks.sort()
ends = sorted(e for s, e, q, n in ks if a.marker in n)
t0, t1 = ends[-a.clips - 1], ends[-1]
win = [k for k in ks if k[0] >= t0 and k[1] <= t1]
span = (t1 - t0) / 1e6
print(f"window {span:.2f} ms = {a.clips} clips ({span / a.clips:.2f} ms per clip), {len(win)} kernels, key {key_q}")
byq = collections.defaultdict(list)
for s, e, q, n in win:
    byq[q].append((s, e, n))
allbusy = union([(s, e) for s, e, _, _ in win]) / 1e6
print(f"any-stream busy {allbusy:.2f} ms ({100 * allbusy / span:.1f} %)")
for q, lst in sorted(byq.items(), key=lambda kv: -len(kv[1])):
    busy = union([(s, e) for s, e, _ in lst]) / 1e6
    tk = collections.Counter()
    for s, e, n in lst:
        tk[short(n)] += (e - s) / 1e6
    top = ", ".join(f"{n} {v:.1f}" for n, v in tk.most_common(4))
    print(f"{key_q} {q}: {len(lst)} kernels, busy {busy:.2f} ms ({100 * busy / span:.1f} %) | {top}")
tot = collections.Counter()
for s, e, q, n in win:
    tot[short(n)] += (e - s) / 1e6
print("kernel time (sum of durations, overlapped):")
for n, v in tot.most_common(a.top):
    print(f"  {v / a.clips:8.3f} ms/clip  {n}")
