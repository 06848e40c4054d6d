#!/bin/bash
# 4x4x4 f64 MFMA form: every-plan test, A/B against the 16x16x4 form, sweep, RMVPE time and tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h; mkdir -p $O
export LD_LIBRARY_PATH=$PWD/rvc-maker_amd/lib:$LD_LIBRARY_PATH
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "conv64 or bordered" > $O/t_ops.log 2>&1 || { tail -30 $O/t_ops.log; exit 1; }
tail -1 $O/t_ops.log
for cfg in; do
  for v in 0_m0 0_m1 15_m0 15_m1; do timeout -k 10 60 scripts/conv64_dbg_$v $cfg >> $O/dbg.log 2>&1 || { echo "dbg $v failed"; cat $O/dbg.log; exit 1; }; done
done
cat $O/dbg.log
timeout -k 10 300 python -u scripts/conv64_sweep.py $O/sweep.json > $O/sweep.log 2>&1 || { tail $O/sweep.log; exit 1; }
grep -c MISMATCH $O/sweep.log; grep "planner\|best" $O/sweep.log
timeout -k 10 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rm.log 2>&1 || { tail $O/rm.log; exit 1; }
tail -1 $O/rm.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rmvpe.py tests/test_gpu_batch.py > $O/t_rm.log 2>&1 || { tail -30 $O/t_rm.log; exit 1; }
tail -1 $O/t_rm.log
