#!/bin/bash
# Is the f64 MFMA rate per SIMD higher when few CUs run (power / clock bound chip-wide)?  MFMA-only loop (C64_DBG 15)
# on 24 .. 768 blocks of the same per-block work.
set -o pipefail
O=gpurun_out/r4n; mkdir -p $O
export LD_LIBRARY_PATH=$PWD/rvc-maker_amd/lib:$LD_LIBRARY_PATH
for cfg in "512 94 4 10 1 1" "512 94 4 10 2 1" "512 94 4 10 4 1" "512 94 4 10 8 1" "512 94 4 10 16 1" "512 94 4 10 32 1"; do
  for v in 15_m0 15_m1; do timeout -k 10 60 scripts/conv64_dbg_$v $cfg >> $O/dbg.log 2>&1 || echo "dbg $v $cfg failed" >> $O/dbg.log; done
done
cat $O/dbg.log
