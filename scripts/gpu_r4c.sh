#!/bin/bash
# f64 RMVPE kernel trace (per grid), then bench and the back-stream A/B (mask default vs unmasked high / normal priority).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rm -o run -- python3 scripts/rmvpe_prof.py f64 5 > $O/rm.log 2>&1 || { echo "rocprof failed"; tail -5 $O/rm.log; exit 1; }
python3 scripts/ktrace_group.py $(ls $O/rm/*/run_kernel_trace.csv $O/rm/run_kernel_trace.csv 2>/dev/null | head -1) 6 > $O/rm_group.txt; cat $O/rm_group.txt
TAG=r4c/ab R=2 VARIANTS="dflt:RVC_X=1 none_hi:RVC_BACK_CU_MASK=none none_norm:RVC_BACK_CU_MASK=none,RVC_AMD_BACK_PRIORITY=0" ./scripts/gpu_ab_env.sh
