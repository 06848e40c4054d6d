#!/bin/bash
# Ablation: the conv engine without its per-chunk barrier (X6_NOBAR=1, wrong results by design) vs default.
set -o pipefail
O=gpurun_out/r4nb; mkdir -p $O
timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 --only 0,1,2,3,4,5,7 > $O/base.log 2>&1 && \
RVC_AMD_LIB=rvc-maker_amd/lib/nobar/librvc_amd.so timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 --only 0,1,2,3,4,5,7 > $O/nobar.log 2>&1
rc=$?; tail -9 $O/base.log; tail -9 $O/nobar.log; exit $rc
