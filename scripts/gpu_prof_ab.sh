#!/bin/bash
# rocprofv3 kernel stats of the per-call bench for lib/base (A) and the in-tree build (B)
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-profab}; mkdir -p $O
for v in A B; do
  if [ $v = A ]; then export RVC_AMD_LIB=$PWD/rvc-maker_amd/lib/base/librvc_amd.so; else unset RVC_AMD_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py --no-stream --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $O/$v.log 2>&1 || { tail -3 $O/$v.log; exit 1; }
  echo "$v $(grep -o '"value": [0-9.]*' $O/$v.log | head -1)"
done
