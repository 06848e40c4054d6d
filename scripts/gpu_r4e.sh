#!/bin/bash
# conv64 debug variants (where the time goes), then the planner sweep and RMVPE f64 time with the fitted model.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
export LD_LIBRARY_PATH=$PWD/rvc-maker_amd/lib:$LD_LIBRARY_PATH
for cfg in "64 752 32 2 4 1" "512 94 4 4 21 1" "16 3008 128 1 1 0"; do
  for d in 0 1 2 3 4 8 12 15; do timeout -k 10 60 scripts/conv64_dbg_$d $cfg >> $O/dbg.log 2>&1 || { echo "dbg $d failed"; cat $O/dbg.log; exit 1; }; done
done
cat $O/dbg.log
timeout -k 10 300 python -u scripts/conv64_sweep.py $O/sweep.json --quick > $O/sweep.log 2>&1 || { tail $O/sweep.log; exit 1; }
grep -v MISMATCH $O/sweep.log | grep -c . ; grep -c MISMATCH $O/sweep.log; grep "planner\|best" $O/sweep.log
timeout -k 10 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rm.log 2>&1 || { tail $O/rm.log; exit 1; }
tail -1 $O/rm.log
