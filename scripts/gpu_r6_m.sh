#!/bin/bash
# round 6: the fused noise source pass under a dirty allocator (scripts/fused_noise_check.py), and the stream tests
# with the split-K reduce off.
set -o pipefail
O=gpurun_out/r6m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/fused_noise_check.py > $O/fn.log 2>&1 || { tail -20 $O/fn.log; exit 1; }
grep -v amdgpu.ids $O/fn.log
for v in sk0:RVC_SPLITK_TILES=0 base:RVC_X=1; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch.py \
    > $O/$name.log 2>&1
  rc=$?
  echo "$name rc=$rc $(grep -E '^FAILED' $O/$name.log | sed 's/.*:://' | cut -c1-60 | tr '\n' ' ')"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop"; exit 1; fi
done
exit 0
