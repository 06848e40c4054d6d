#!/bin/bash
# mixed fp32 policy: op/resblock tests, pipeline precision check, bench A/B vs fp32x6
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_resblock.py tests/test_gpu_synth.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/mix_test.log 2>&1; rc=$?
tail -4 gpurun_out/mix_test.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/mix_test.log | head -10; exit $rc; }
timeout -k 10 300 python scripts/prec_check.py > gpurun_out/prec.log 2>&1; tail -5 gpurun_out/prec.log
for prec in fp32x6 fp32 fp32x6 fp32; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --precision $prec > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('$prec', d['value'], d['ms_per_step'], d.get('per_call'), d['roofline']['frac'], d['roofline']['achieved'])"
done
