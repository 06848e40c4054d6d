#!/bin/bash
# A/B: split-K target grid (RVC_SPLITK_TILES: 512 default, 128, 0 = never split) on the clip stream.
set -o pipefail
O=gpurun_out/r4s; mkdir -p $O
run() { RVC_SPLITK_TILES=$2 timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/$1.log 2>&1; }
run b1 512 && run z1 0 && run q1 128 && run b2 512 && run z2 0 && run q2 128
rc=$?
for f in b1 z1 q1 b2 z2 q2; do grep '"metric"' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['per_call'])"; done
exit $rc
