#!/bin/bash
# round 5: RMVPE alone (30 s clip), f64 and fp32sa -- kernel trace for the per-level time split
set -o pipefail
O=gpurun_out/r5m; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for pr in f64 fp32sa; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$pr -o run -- python3 scripts/rmvpe_prof.py $pr 3 > $O/$pr.log 2>&1 || { tail -20 $O/$pr.log; exit 1; }
tail -2 $O/$pr.log
done
find $O -name "*.csv" | head
