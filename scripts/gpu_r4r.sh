#!/bin/bash
set -o pipefail
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 600 python -u scripts/conv64_sweep.py $O/sweep_direct.json --direct > $O/sweep.log 2>&1 || { tail $O/sweep.log; exit 1; }
grep -c MISMATCH $O/sweep.log; grep "planner\|best" $O/sweep.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "wino or conv64 or bordered" > $O/t_ops.log 2>&1 || { tail -30 $O/t_ops.log; exit 1; }
tail -1 $O/t_ops.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/rm -o run -- python3 scripts/rmvpe_prof.py f64 5 > $O/rm.log 2>&1 || { tail -5 $O/rm.log; exit 1; }
python3 scripts/ktrace_group.py $O/rm/run_kernel_trace.csv 6 wino > $O/group_wino.txt; cat $O/group_wino.txt
timeout -k 10 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rm2.log 2>&1 && tail -1 $O/rm2.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rmvpe.py tests/test_gpu_native.py tests/test_gpu_batch.py > $O/t_rm.log 2>&1 || { tail -30 $O/t_rm.log; exit 1; }
tail -1 $O/t_rm.log
TAG=r4r/ab R=2 VARIANTS="wino:RVC_X=1 unfused_only:RVC_RMVPE_WINO=2 off:RVC_RMVPE_WINO=0 gru8:RVC_BIGRU64_WG=8" ./scripts/gpu_ab_env.sh
RVC_BIGRU64_WG=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py -k bigru > $O/t_gru8.log 2>&1 || { tail -30 $O/t_gru8.log; exit 1; }
tail -1 $O/t_gru8.log
