#!/bin/bash
# round 6, ninth GPU pass: the C = 32 pair's two R buffers (tile k - 1's outputs stored after S1(k), RVC_RB_YLDS=2);
# the touched suites, per-tile stamps of both output orders, an interleaved A/B, the default bench line (12 clips).
set -o pipefail
O=gpurun_out/r6i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest --maxfail=20 -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_resblock.py tests/test_gpu_synth.py tests/test_gpu_native.py tests/test_gpu_pipeline.py \
  tests/test_gpu_batch.py > $O/tests.log 2>&1
rc=$?
tail -30 $O/tests.log | grep -v "^\.\.\.\." | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stop"; exit 1; fi
grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/tests.log && { echo "GPU fault: stop"; exit 1; }
for y in 2 1; do
  RVC_RB_YLDS=$y RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 200 python -u scripts/rb_stamps.py \
    --out $O/rb_stamps_y$y.json > $O/rb_stamps_y$y.log 2>&1 || { tail -5 $O/rb_stamps_y$y.log; exit 1; }
  grep -E "^c32" $O/rb_stamps_y$y.log | cut -c1-260
done
TAG=r6i/ab VARIANTS="new:RVC_X=1 ylds1:RVC_RB_YLDS=1" R=3 bash scripts/gpu_ab_env.sh || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python3 -c "
import json; d = json.loads(open('$O/bench.json').read()); r = d['roofline']
print('value', d['value'], 'steps', d['steps'], 'per_call', d['per_call'], 'frac', r['frac'])
"
