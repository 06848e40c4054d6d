#!/bin/bash
set -u
mkdir -p gpurun_out
for bn in 0 2; do
  for prec in fp32x6 f16x3; do
    RVC_X6_BN256=$bn timeout -k 10 200 python scripts/conv_bench.py --precision $prec --check --only 0,1,2,3,4 > gpurun_out/cb_$bn$prec.log 2>&1 || { tail gpurun_out/cb_$bn$prec.log; exit 1; }
    echo "== BN256=$bn $prec"; grep "C=\|total" gpurun_out/cb_$bn$prec.log | cut -c1-100
  done
done
RVC_X6_BN256=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 200 --timeout-method thread -k conv > gpurun_out/bn_test.log 2>&1; tail -2 gpurun_out/bn_test.log
for bn in 0 1 2 0 1 2; do
  RVC_X6_BN256=$bn timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-per-call > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('bn256=$bn', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
