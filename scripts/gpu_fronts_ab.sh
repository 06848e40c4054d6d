#!/bin/bash
# Clip stream with 1 vs 2 alternating front pipelines (RVC_STREAM_FRONTS) and the hardware-queue count.
set -u
mkdir -p gpurun_out
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps ${STEPS:-12} --warmup 2 --no-cpu-baseline --no-per-call ${MODE:-} > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('$label', d['value'], d['ms_per_step'])"
}
timeout -k 10 300 env GPU_MAX_HW_QUEUES=8 RVC_STREAM_FRONTS=2 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread -k stream > gpurun_out/fronts_test.log 2>&1 || { tail -30 gpurun_out/fronts_test.log; exit 1; }
tail -1 gpurun_out/fronts_test.log
run default X=1
run q8_f1 GPU_MAX_HW_QUEUES=8
run q8_f2 GPU_MAX_HW_QUEUES=8 RVC_STREAM_FRONTS=2
run q8_f3 GPU_MAX_HW_QUEUES=8 RVC_STREAM_FRONTS=3
run default X=1
run q8_f2 GPU_MAX_HW_QUEUES=8 RVC_STREAM_FRONTS=2
