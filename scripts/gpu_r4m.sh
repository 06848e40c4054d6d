#!/bin/bash
# 16x16x4 (m0) vs 4x4x4 (m1) f64 MFMA form in the conv engine, plain event timing, several plans.
set -o pipefail
O=gpurun_out/r4m; mkdir -p $O
export LD_LIBRARY_PATH=$PWD/rvc-maker_amd/lib:$LD_LIBRARY_PATH
for cfg in "128 376 16 9 4 1" "128 376 16 9 1 1" "64 752 32 9 2 1" "512 94 4 10 21 1" "512 94 4 9 16 1" "16 3008 128 1 1 0" "16 3008 128 8 1 0" "256 188 8 9 8 1"; do
  for v in 0_m0 0_m1 15_m0 15_m1; do timeout -k 10 60 scripts/conv64_dbg_$v $cfg >> $O/dbg.log 2>&1 || echo "dbg $v $cfg failed" >> $O/dbg.log; done
done
cat $O/dbg.log
