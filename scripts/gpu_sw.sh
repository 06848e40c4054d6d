#!/bin/bash
# swizzle check: fused + conv tests, conv_bench suite, rb_bench, bench
set -u
OUT=gpurun_out/sw; mkdir -p $OUT
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-3} | cut -c1-400; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
run t_ops 400 python -u -m pytest tests/test_gpu_resblock.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread
TAILN=14 run rb 200 python -u scripts/rb_bench.py
TAILN=12 run cb 200 python -u scripts/conv_bench.py --reps 5
run bench 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
echo all ok
