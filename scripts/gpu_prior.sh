#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_pm.py tests/test_gpu_synth.py tests/test_gpu_pipeline.py tests/test_gpu_convert.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/prior_test.log 2>&1; rc=$?
tail -3 gpurun_out/prior_test.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/prior_test.log | head; exit $rc; }
for mode in front back front back; do
  RVC_AMD_STREAM_PRIOR=$mode timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-per-call > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('prior=$mode', d['value'], d['ms_per_step'])"
done
