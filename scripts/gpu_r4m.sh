#!/bin/bash
# A/B (round 4, a since-removed switch): split factor from a round-quantised cost (RVC_SPLITK_MODEL=1) vs ceil(target / tiles).
set -o pipefail
O=gpurun_out/r4m; mkdir -p $O
a() { timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/$1.log 2>&1; }
m() { RVC_SPLITK_MODEL=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/$1.log 2>&1; }
RVC_SPLITK_MODEL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_contentvec.py > $O/tests.log 2>&1; tail -2 $O/tests.log
a a1 && m m1 && a a2 && m m2 && a a3 && m m3
rc=$?
for f in a1 m1 a2 m2 a3 m3; do grep '"metric"' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['per_call'])"; done
exit $rc
