#!/bin/bash
# A/B of two library builds (default vs lib/b) on conv shapes and the bench, same box
set -u
mkdir -p gpurun_out
B=rvc-maker_amd/lib/b/librvc_amd.so
for prec in fp32x6 f16x3; do
  timeout -k 10 200 python scripts/conv_bench.py --precision $prec > gpurun_out/cbA.log 2>&1 || { tail gpurun_out/cbA.log; exit 1; }
  RVC_AMD_LIB=$B timeout -k 10 200 python scripts/conv_bench.py --precision $prec > gpurun_out/cbB.log 2>&1 || { tail gpurun_out/cbB.log; exit 1; }
  echo "== $prec  A (new) | B"; paste <(grep "C=\|total" gpurun_out/cbA.log | cut -c1-62) <(grep "C=\|total" gpurun_out/cbB.log | cut -c27-62)
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_resblock.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ab_test.log 2>&1; tail -2 gpurun_out/ab_test.log
for lib in "" $B "" $B; do
  RVC_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('lib=$lib', d['value'], d['ms_per_step'], d.get('per_call'), d['roofline']['frac'])"
done
