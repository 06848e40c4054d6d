#!/bin/bash
# Re-measure two round-3 conv engine defaults in the round-4 clip stream: k-order stagger (RVC_X6_ROT=1) and the
# XCD-aware tile order off (RVC_X6_XCD=0), each against the default, alternated.
set -o pipefail
O=gpurun_out/r4env; mkdir -p $O
run() { env $2 timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/$1.log 2>&1; }
run d1 X=0 && run r1 RVC_X6_ROT=1 && run x1 RVC_X6_XCD=0 && run d2 X=0 && run r2 RVC_X6_ROT=1 && run x2 RVC_X6_XCD=0
rc=$?
for f in d1 r1 x1 d2 r2 x2; do grep '"metric"' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['per_call'])"; done
exit $rc
