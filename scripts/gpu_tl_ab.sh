#!/bin/bash
# clip-stream timelines (rocprofv3 kernel trace) for lib/base (A) and the in-tree build (B)
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tlab}; mkdir -p $O
for v in A B; do
  if [ $v = A ]; then export RVC_AMD_LIB=$PWD/rvc-maker_amd/lib/base/librvc_amd.so; else unset RVC_AMD_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-per-call --no-roofline > $O/$v.log 2>&1 || { tail -3 $O/$v.log; exit 1; }
  f=$(find $O/$v -name "*kernel_trace.csv" | head -1)
  python3 scripts/timeline.py "$f" > $O/tl_$v.txt 2>&1
  echo "== $v $(grep -o '"value": [0-9.]*' $O/$v.log | head -1)"; head -8 $O/tl_$v.txt | cut -c1-250
  rm -f "$f"
done
