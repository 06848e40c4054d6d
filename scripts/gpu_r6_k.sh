#!/bin/bash
# round 6: is the stream / batch bit-identity failure of r6i order-dependent?  tests/test_gpu_batch.py alone, then after
# each suite that ran before it in r6i (one process each).
set -o pipefail
O=gpurun_out/r6k; mkdir -p $O
export TMPDIR=/tmp
B=tests/test_gpu_batch.py
for v in alone: pipeline:tests/test_gpu_pipeline.py native:tests/test_gpu_native.py synth:tests/test_gpu_synth.py \
         resblock:tests/test_gpu_resblock.py; do
  name=${v%%:*}; pre=${v#*:}
  timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu $pre $B > $O/$name.log 2>&1
  rc=$?
  echo "$name rc=$rc $(grep -E '^FAILED' $O/$name.log | cut -c1-100 | tr '\n' ' ') $(tail -1 $O/$name.log | cut -c1-80)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop"; exit 1; fi
  grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/$name.log && { echo "GPU fault: stop"; exit 1; }
done
exit 0
