#!/bin/bash
# Interleaved bench A/B of two library builds on one box: lib/base (A) against the in-tree build (B)
set -u
O=gpurun_out/${TAG:-ablib}; mkdir -p $O
A=$PWD/rvc-maker_amd/lib/base/librvc_amd.so
for r in 1 2 3; do
  for v in ${ORDER:-A B}; do
    if [ $v = A ]; then export RVC_AMD_LIB=$A; else unset RVC_AMD_LIB; fi
    if [ $v = B ]; then export ${BENV:-RVC_NOTHING=0}; else unset ${BENV%%=*}; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --no-per-call --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS:-} > $O/b_$v$r.log 2>&1 || { tail -3 $O/b_$v$r.log; exit 1; }
    echo "$v$r $(grep -o '"value": [0-9.]*' $O/b_$v$r.log | head -1)"
  done
done
