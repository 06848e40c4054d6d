#!/bin/bash
# f64 conv planner: every-plan test, the RMVPE shape sweep, RMVPE f64 time, the f64 RMVPE tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
step() { local t=$1; shift; echo "== $*"; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
true
step 300 python -u scripts/conv64_sweep.py $O/sweep.json > $O/sweep.log 2>&1; cat $O/sweep.log
step 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rm.log 2>&1; tail -1 $O/rm.log
step 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rmvpe.py tests/test_gpu_native.py tests/test_gpu_batch.py > $O/t_rm.log 2>&1; tail -3 $O/t_rm.log
