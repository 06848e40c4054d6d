#!/bin/bash
# Clip-stream priority variants on one GPU (same box).
set -u
mkdir -p gpurun_out
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-per-call ${MODE:-} > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('$label', d['value'], d['ms_per_step'])"
}
run default X=1
run fside_hi RVC_AMD_FSIDE_PRIORITY=-1
run fronts_hi RVC_AMD_FSIDE_PRIORITY=-1 RVC_AMD_FRONT_PRIORITY=-1
run back_norm_fside_hi RVC_AMD_FSIDE_PRIORITY=-1 RVC_AMD_BACK_PRIORITY=0
run default X=1
run fside_hi RVC_AMD_FSIDE_PRIORITY=-1
