#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4y; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/rm -o run -- python3 scripts/rmvpe_prof.py f64 5 > $O/rm.log 2>&1 || { tail -5 $O/rm.log; exit 1; }
python3 scripts/ktrace_group.py $O/rm/run_kernel_trace.csv 6 > $O/group.txt; head -42 $O/group.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench.py > $O/t_bench.log 2>&1 || { tail -30 $O/t_bench.log; exit 1; }
tail -1 $O/t_bench.log
