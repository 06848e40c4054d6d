#!/bin/bash
# A/B: split-K target grid RVC_SPLITK_TILES in {512, 256, 128, 64} on the clip stream, twice.
set -o pipefail
O=gpurun_out/r4s2; mkdir -p $O
run() { RVC_SPLITK_TILES=$2 timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/$1.log 2>&1; }
run a1 512 && run b1 256 && run c1 128 && run d1 64 && run a2 512 && run b2 256 && run c2 128 && run d2 64
rc=$?
for f in a1 b1 c1 d1 a2 b2 c2 d2; do grep '"metric"' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['per_call'])"; done
exit $rc
