#!/bin/bash
# BASELINE.json configs on one GPU: headline (configs[1]), cfg 3 shape (64 x 10 s, bf16, index 0.75),
# cfg 5 shape (40k, crepe-full, bf16, hipGraph chunk loop); then a rocprofv3 kernel-stats pass.
set -u
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 600 python bench.py "$@" > gpurun_out/cfg_$tag.log 2>&1
  local rc=$?
  echo "== $tag rc=$rc"; tail -1 gpurun_out/cfg_$tag.log | cut -c1-330
  return $rc
}
run headline --steps 10 --warmup 2 || exit $?
run headline_graph --steps 10 --warmup 2 --graph --no-cpu-baseline || exit $?
run cfg3 --steps 2 --warmup 1 --chunks 64 --seconds 10 --precision bf16 --index-rate 0.75 --no-cpu-baseline || exit $?
run cfg3_fp32 --steps 2 --warmup 1 --chunks 64 --seconds 10 --index-rate 0.75 --no-cpu-baseline || exit $?
run cfg5 --steps 2 --warmup 1 --chunks 4 --sr 40000 --f0 crepe-full --precision bf16 --graph --no-cpu-baseline || exit $?
bash scripts/gpu_prof.sh r1 || exit $?
