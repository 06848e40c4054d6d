#!/bin/bash
# Winograd (unfused, per-thread input transform): tests, RMVPE time, bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "wino or conv64 or bordered" > $O/t_ops.log 2>&1 || { tail -30 $O/t_ops.log; exit 1; }
tail -1 $O/t_ops.log
timeout -k 10 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rm.log 2>&1 || { tail $O/rm.log; exit 1; }
tail -1 $O/rm.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rmvpe.py tests/test_gpu_native.py tests/test_gpu_batch.py > $O/t_rm.log 2>&1 || { tail -30 $O/t_rm.log; exit 1; }
tail -1 $O/t_rm.log
TAG=r4s/ab R=2 VARIANTS="wino:RVC_X=1 off:RVC_RMVPE_WINO=0 fronts2q8:RVC_STREAM_FRONTS=2,GPU_MAX_HW_QUEUES=8 q8:GPU_MAX_HW_QUEUES=8" ./scripts/gpu_ab_env.sh
