#!/bin/bash
set -u
mkdir -p gpurun_out
for x in 1 0 1 0; do
  RVC_GRU_XCD=$x timeout -k 10 200 python scripts/micro.py bigru > gpurun_out/gru.log 2>&1 || { tail gpurun_out/gru.log; exit 1; }
  echo "xcd=$x $(grep B= gpurun_out/gru.log | head -1)"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_rmvpe.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gru_test.log 2>&1; tail -2 gpurun_out/gru_test.log
for x in 1 0 1 0; do
  RVC_GRU_XCD=$x timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-per-call > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('xcd=$x', d['value'], d['ms_per_step'])"
done
