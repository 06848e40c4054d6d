#!/bin/bash
# round 6: the fused noise pass off by default (stream use-after-free exposure, r6j-r6p); ContentVec's split-fp16
# attention with 32 queries per wave; the rel-v band kernel on LDS-staged Q / K.  Suites, an A/B and the bench line.
set -o pipefail
O=gpurun_out/r6q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest --maxfail=20 -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_batch.py tests/test_gpu_amax.py tests/test_gpu_ops.py tests/test_gpu_contentvec.py tests/test_gpu_synth.py \
  tests/test_gpu_native.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1
rc=$?
tail -30 $O/tests.log | grep -v "^\.\.\.\." | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stop"; exit 1; fi
grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/tests.log && { echo "GPU fault: stop"; exit 1; }
timeout -k 10 300 python -u scripts/synth_stage_time.py --out $O/synth_stages.json base ATTN_F16=0 > $O/ss.log 2>&1 || { tail -5 $O/ss.log; exit 1; }
grep -v amdgpu.ids $O/ss.log
TAG=r6q/ab VARIANTS="new:RVC_X=1 attn0:RVC_AMD_ATTN_F16=0 noise1:RVC_AMD_FUSED_NOISE=1" R=2 bash scripts/gpu_ab_env.sh || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python3 -c "
import json; d = json.loads(open('$O/bench.json').read()); r = d['roofline']
print('value', d['value'], 'steps', d['steps'], 'per_call', d['per_call'], 'frac', r['frac'])
for k, v in (r.get('families') or {}).items(): print(' ', k, v.get('achieved'), v.get('unit'), 'frac', v.get('frac'), 'ms', v.get('kernel_ms'))
"
