#!/bin/bash
# conv64 chunk depth KC 16 vs 32 over plans (split-K 1 isolates the conv kernel from the reduce).
set -o pipefail
O=gpurun_out/r4g; mkdir -p $O
export LD_LIBRARY_PATH=$PWD/rvc-maker_amd/lib:$LD_LIBRARY_PATH
for cfg in "64 752 32 2 4 1" "64 752 32 2 1 1" "64 752 32 3 1 1" "512 94 4 4 21 1" "512 94 4 4 8 1" "16 3008 128 1 1 0" "128 376 16 2 8 1" "128 376 16 3 2 1" "256 188 8 3 8 1" "32 1504 64 3 1 1"; do
  for v in kc16 kc32; do timeout -k 10 60 scripts/conv64_dbg_$v $cfg >> $O/dbg.log 2>&1 || echo "dbg $v $cfg refused" >> $O/dbg.log; done
done
cat $O/dbg.log
