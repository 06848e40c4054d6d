#!/bin/bash
# A/B: the fused 128-channel ResBlock pair (RVC_AMD_FUSED_RB128=1) vs two launches, with the pinned B reads.
set -o pipefail
O=gpurun_out/r4rb128; mkdir -p $O
a() { timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/$1.log 2>&1; }
f() { RVC_AMD_FUSED_RB128=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/$1.log 2>&1; }
a a1 && f f1 && a a2 && f f2
rc=$?
for x in a1 f1 a2 f2; do grep '"metric"' $O/$x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$x', d['value'], d['per_call'])"; done
exit $rc
