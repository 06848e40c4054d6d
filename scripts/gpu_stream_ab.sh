#!/bin/bash
# Clip-stream variants on one GPU (same box).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/stream_test.log 2>&1 || { tail -30 gpurun_out/stream_test.log; exit 1; }
tail -2 gpurun_out/stream_test.log
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup ${WARM:-2} --no-cpu-baseline ${MODE:-} > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('$label', d['value'], d['ms_per_step'], d.get('per_call'), d['roofline']['frac'])"
}
WARM=1 STEPS=2 MODE="--chunks 64 --seconds 10 --index-rate 0.75 --precision bf16x3 --batch 16" run cfg3_stream_b16 X=1
WARM=1 STEPS=2 MODE="--chunks 64 --seconds 10 --index-rate 0.75 --precision bf16x3 --batch 8" run cfg3_stream_b8 X=1
WARM=1 STEPS=2 MODE="--chunks 64 --seconds 10 --index-rate 0.75 --precision bf16x3 --batch 4" run cfg3_stream_b4 X=1
