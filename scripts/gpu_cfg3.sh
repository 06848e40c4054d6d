#!/bin/bash
# cfg3 A/B: unbatched vs batched 64 x 10 s chunks (bf16x3, index 0.75), the 30 s bf16x3 clip, and a rocprof of the batched step
set -u
OUT=gpurun_out/cfg3; mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids $OUT/$name.log | tail -1 | cut -c1-330; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
C3="--chunks 64 --seconds 10 --precision bf16x3 --index-rate 0.75 --no-cpu-baseline"
run unbatched 300 python bench.py --steps 2 --warmup 1 $C3
run b16 300 python bench.py --steps 2 --warmup 1 $C3 --batch 16
run b32 300 python bench.py --steps 2 --warmup 1 $C3 --batch 32
run clip30 300 python bench.py --steps 5 --warmup 2 --precision bf16x3 --no-cpu-baseline
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 1 --warmup 1 $C3 --batch 16
echo all ok
