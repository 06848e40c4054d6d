#!/bin/bash
# A/B on one box: new defaults (split-K target 256, 128-wide split-fp16 tiles when the 256-wide grid
# quantises worse) vs the previous ones (RVC_SPLITK_TILES=512 RVC_X6_BN256=3).
set -o pipefail
O=gpurun_out/r4t; mkdir -p $O
old() { RVC_SPLITK_TILES=512 RVC_X6_BN256=3 timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/$1.log 2>&1; }
new() { timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/$1.log 2>&1; }
timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 --check > $O/conv.log 2>&1 && \
old o1 && new n1 && old o2 && new n2 && old o3 && new n3
rc=$?; grep "C=\|total" $O/conv.log
for f in o1 n1 o2 n2 o3 n3; do grep '"metric"' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['per_call'])"; done
exit $rc
