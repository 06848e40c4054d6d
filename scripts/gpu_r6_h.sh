#!/bin/bash
# round 6, eighth GPU pass: ContentVec layer 0 over more workgroups (64-frame stat tiles, channel-group apply), the
# bench's attention families on the split-fp16 kernels; the touched suites, the environment switches re-measured on
# the round's kernels (interleaved A/B, one box) and the default bench line.
set -o pipefail
O=gpurun_out/r6h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest --maxfail=20 -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py tests/test_gpu_amax.py tests/test_gpu_contentvec.py tests/test_gpu_native.py \
  tests/test_gpu_pipeline.py tests/test_gpu_bench.py > $O/tests.log 2>&1
rc=$?
tail -30 $O/tests.log | grep -v "^\.\.\.\." | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stop"; exit 1; fi
grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/tests.log && { echo "GPU fault: stop"; exit 1; }
TAG=r6h/ab VARIANTS="new:RVC_X=1 noise0:RVC_AMD_FUSED_NOISE=0 sk512:RVC_SPLITK_TILES=512 mxwg8:RVC_BIGRU64_MXWG=8 attn0:RVC_AMD_ATTN_F16=0 swz0:RVC_X6_SWZ=0 grp0:RVC_X6_GROUPED=0" R=2 bash scripts/gpu_ab_env.sh || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python3 -c "
import json; d = json.loads(open('$O/bench.json').read()); r = d['roofline']
print('value', d['value'], 'per_call', d['per_call'], 'frac', r['frac'])
for k, v in (r.get('families') or {}).items(): print(' ', k, v.get('achieved'), v.get('unit'), 'frac', v.get('frac'), 'ms', v.get('kernel_ms'))
"
