#!/bin/bash
# Ablations of the split-fp16 128 x 256 conv (RVC_CONV_ABLATIONS=1 build; wrong results by design):
# RVC_CONV_DEBUG 1 = no epilogue, 2 = no MFMA, 4 = no input loads, sums thereof.
set -o pipefail
O=gpurun_out/r4abl; mkdir -p $O
export RVC_AMD_LIB=rvc-maker_amd/lib/abl/librvc_amd.so
for d in 0 1 2 4 3 5 6 7; do
  RVC_CONV_DEBUG=$d timeout -k 10 200 python -u scripts/conv_bench.py --reps 10 --only 0,2,4 > $O/d$d.log 2>&1 || exit 1
  echo "dbg=$d"; grep "C=" $O/d$d.log
done
