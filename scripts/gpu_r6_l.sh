#!/bin/bash
# round 6: tests/test_gpu_batch.py as a module (its stream tests fail after the module's earlier tests, r6k) under each
# feature switch off, twice each.
set -o pipefail
O=gpurun_out/r6l; mkdir -p $O
export TMPDIR=/tmp
B=tests/test_gpu_batch.py
for v in base:RVC_X=1 ylds0:RVC_RB_YLDS=0 wide0:RVC_RB_WIDE64=0 noise0:RVC_AMD_FUSED_NOISE=0 grp0:RVC_X6_GROUPED=0 \
         attn0:RVC_AMD_ATTN_F16=0 swz0:RVC_X6_SWZ=0 fe0:RVC_AMD_FE_AMAX=0 s2:RVC_AMD_AMAX_S2=0 amax0:RVC_AMD_AMAX=0 \
         cv0:RVC_AMD_CV_AMAX=0 f16all0:RVC_AMD_AMAX_F16ALL=0 ups0:RVC_AMD_AMAX_UPS=0; do
  for r in 1 2; do
    name=${v%%:*}; envs=${v#*:}
    env $(echo $envs | tr ',' ' ') timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu $B \
      > $O/${name}_$r.log 2>&1
    rc=$?
    echo "$name#$r rc=$rc $(grep -E '^FAILED' $O/${name}_$r.log | sed 's/.*:://' | cut -c1-60 | tr '\n' ' ') $(grep -o 'AssertionError: ([0-9], [0-9.e-]*)' $O/${name}_$r.log | tr '\n' ' ')"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop"; exit 1; fi
    grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/${name}_$r.log && { echo "GPU fault: stop"; exit 1; }
  done
done
exit 0
