#!/bin/bash
# A/B: 128 x 256 vs 128 x 128 tiles for the split-fp16 convs (RVC_X6_BN256=0), per shape, twice.
set -o pipefail
O=gpurun_out/r4bn; mkdir -p $O
timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 > $O/a1.log 2>&1 && \
RVC_X6_BN256=0 timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 > $O/b1.log 2>&1 && \
timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 > $O/a2.log 2>&1 && \
RVC_X6_BN256=0 timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 > $O/b2.log 2>&1
rc=$?; for f in a1 b1 a2 b2; do echo == $f; grep "C=\|total" $O/$f.log; done; exit $rc
