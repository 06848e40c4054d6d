#!/bin/bash
# 36-deep channel-aligned chunks: every-plan test, direct-shape sweep, RMVPE time, clip stream A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "wino or conv64 or bordered" > $O/t_ops.log 2>&1 || { tail -30 $O/t_ops.log; exit 1; }
tail -1 $O/t_ops.log
timeout -k 10 600 python -u scripts/conv64_sweep.py $O/sweep_direct.json --direct > $O/sweep.log 2>&1 || { tail $O/sweep.log; exit 1; }
grep -c MISMATCH $O/sweep.log; grep "planner\|best" $O/sweep.log
for v in 1 0; do RVC_C64_KC36=$v timeout -k 10 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rm$v.log 2>&1 || { tail $O/rm$v.log; exit 1; }; echo "kc36=$v $(tail -1 $O/rm$v.log)"; done
TAG=r4w/ab R=2 VARIANTS="kc36:RVC_X=1 nokc36:RVC_C64_KC36=0" ./scripts/gpu_ab_env.sh
