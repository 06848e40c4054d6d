#!/bin/bash
# split-fp16 engine: unit tests, conv shapes (speed + check), pipeline error per precision, bench A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 120 --timeout-method thread -k "f16x3 or reduced or conv1d" > gpurun_out/f16_test.log 2>&1; rc=$?
tail -15 gpurun_out/f16_test.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python scripts/conv_bench.py --precision fp32 > gpurun_out/cb_fp32.log 2>&1 || { tail gpurun_out/cb_fp32.log; exit 1; }
timeout -k 10 200 python scripts/conv_bench.py --precision f16x3 --check > gpurun_out/cb_f16.log 2>&1; crc=$?
paste <(cut -c1-60 gpurun_out/cb_fp32.log) <(cut -c24-200 gpurun_out/cb_f16.log)
[ $crc -ne 0 ] && exit $crc
timeout -k 10 300 python scripts/prec_check.py > gpurun_out/prec.log 2>&1; cat gpurun_out/prec.log | tail -5
for prec in fp32 f16x3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --precision $prec > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('$prec', d['value'], d['ms_per_step'], d.get('per_call'), d['roofline']['frac'], d['roofline']['achieved'])"
done
