#!/bin/bash
# round 6: which switch makes pipeline_device_stream differ from the per-call / batch forms (tests/test_gpu_batch.py
# failed in r6i) -- the batched stream test under each feature switch off, one process per setting.
set -o pipefail
O=gpurun_out/r6j; mkdir -p $O
export TMPDIR=/tmp
T=tests/test_gpu_batch.py::test_batched_stream_bit_identical_to_batch
for v in base:RVC_X=1 ylds1:RVC_RB_YLDS=1 ylds0:RVC_RB_YLDS=0 wide0:RVC_RB_WIDE64=0 noise0:RVC_AMD_FUSED_NOISE=0 \
         grp0:RVC_X6_GROUPED=0 attn0:RVC_AMD_ATTN_F16=0 swz0:RVC_X6_SWZ=0 fe0:RVC_AMD_FE_AMAX=0 s2:RVC_AMD_AMAX_S2=0 \
         amax0:RVC_AMD_AMAX=0 cv0:RVC_AMD_CV_AMAX=0; do
  name=${v%%:*}; envs=${v#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 240 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $T \
    > $O/$name.log 2>&1
  rc=$?
  echo "$name rc=$rc $(grep -o 'AssertionError: ([0-9], [0-9.e-]*)' $O/$name.log | head -1) $(tail -1 $O/$name.log | cut -c1-80)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop"; exit 1; fi
  grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/$name.log && { echo "GPU fault: stop"; exit 1; }
done
exit 0
