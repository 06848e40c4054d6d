#!/bin/bash
# Clip stream: parity tests (stream, graph), then the default bench (stream + per_call) and --no-stream.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_graph.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/stream_test.log 2>&1 || { tail -30 gpurun_out/stream_test.log; exit 1; }
tail -3 gpurun_out/stream_test.log
for mode in "" "--no-stream" ""; do
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline $mode ${EXTRA:-} > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('$mode', d['value'], d['ms_per_step'], d.get('per_call'), d['roofline']['frac'])"
done
