#!/bin/bash
# round 6: the fused source pass under the clip stream, diagnosis variants (RVC_SRC_DBG: 1 no |max| publish, 2 per-wave
# publish (no static LDS), 3 1 KB of extra LDS, 4 host sync after the pass) -- scripts/stream_diff.py, 2 reps each.
set -o pipefail
O=gpurun_out/r6o; mkdir -p $O
export TMPDIR=/tmp
for d in 0 1 2 3 4; do
  RVC_SRC_DBG=$d timeout -k 10 300 python -u scripts/stream_diff.py --reps 2 > $O/sd_$d.log 2>&1 || { tail -20 $O/sd_$d.log; exit 1; }
  echo "== RVC_SRC_DBG=$d"; grep -E "^rep" $O/sd_$d.log | cut -c1-150
done
