#!/bin/bash
# LayerNorm: LDS-tile form (RVC_LN_REG=0) vs register-resident form (default); parity, microbench, bench A/B.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_norm.py tests/test_gpu_contentvec.py tests/test_gpu_synth.py tests/test_gpu_native.py tests/test_gpu_pipeline.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ln_test.log 2>&1 || { tail -30 gpurun_out/ln_test.log; exit 1; }
tail -1 gpurun_out/ln_test.log
for v in 0 1; do RVC_LN_REG=$v timeout -k 10 120 python scripts/micro.py norms 2>&1 | grep -v amdgpu.ids | sed "s/^/reg=$v /"; done
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 12 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('$label', d['value'], d['ms_per_step'], 'per_call', d['per_call'])"
}
run reg1 RVC_LN_REG=1
run reg0 RVC_LN_REG=0
run reg1 RVC_LN_REG=1
run reg0 RVC_LN_REG=0
