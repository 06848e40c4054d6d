#!/bin/bash
# round 5: the hot conv's PMC on the production path (the |max| cell: fast-only split-fp16 loader kernel) and the
# per-shape timings with and without the cell
set -o pipefail
O=gpurun_out/r5y; mkdir -p $O
export TMPDIR=/tmp
for a in "" "--amax"; do
timeout -k 10 300 python3 -u scripts/conv_bench.py --precision fp32 $a > $O/cb$a.log 2>&1 || { tail -20 $O/cb$a.log; exit 1; }
echo "== conv_bench $a"; grep -v -i warn $O/cb$a.log | grep -v amdgpu.ids
done
TAG=r5y/pmc CB_ARGS="--amax" bash scripts/gpu_pmc_hot.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
tail -4 $O/pmc.log
