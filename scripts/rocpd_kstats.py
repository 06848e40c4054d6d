"""Per-kernel time from a rocprofv3 results database (run_results.db): total ms per pass, calls per pass, mean us,
and the wall span of the traced dispatches.

    python scripts/rocpd_kstats.py gpurun_out/x/run_results.db PASSES [top]
"""
import re
import sqlite3
import sys
from collections import defaultdict


def dispatches(db):
    c = sqlite3.connect(db)
    q = ("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    return [(re.sub(r"\(anonymous namespace\)::", "", n).split("(")[0][:80], a, b) for n, a, b in c.execute(q)]


def main():
    db, passes = sys.argv[1], float(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = dispatches(db)
    acc = defaultdict(list)
    for n, a, b in rows:
        acc[n].append((b - a) / 1e3)
    tot = sum(sum(v) for v in acc.values())
    print(f"{len(rows) / passes:.0f} dispatches per pass, kernel time {tot / passes / 1e3:.2f} ms per pass, "
          f"span {(rows[-1][2] - rows[0][1]) / 1e6 / passes:.2f} ms per pass")
    for n, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{sum(v) / passes / 1e3:7.3f} ms {len(v) / passes:6.1f} calls {sum(v) / len(v):8.1f} us  {n}")


if __name__ == "__main__":
    main()
