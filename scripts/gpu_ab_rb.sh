#!/bin/bash
# A/B of the fused ResBlock pair's weight prefetch depth (RB_PD2, split-fp16 / 3-pass builds in lib/pdN)
set -u
O=gpurun_out/${TAG:-abrb}; mkdir -p $O
for v in main pd4 pd6; do
  L=rvc-maker_amd/lib/librvc_amd.so; [ $v != main ] && L=rvc-maker_amd/lib/$v/librvc_amd.so
  RVC_AMD_LIB=$PWD/$L timeout -k 10 300 python -u scripts/rb_bench.py --reps 5 > $O/rb_$v.log 2>&1 || { tail -5 $O/rb_$v.log; exit 1; }
  echo "== $v"; tail -14 $O/rb_$v.log
done
