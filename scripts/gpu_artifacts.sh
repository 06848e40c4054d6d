#!/bin/bash
# Round artifacts: the default bench line, rocprof kernel stats of the per-call bench (the roofline probe's
# setting), PMC HBM traffic, and the clip-stream timeline.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/art
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/art/bench.log 2>&1; rc=$?
echo "bench exit=$rc" >> gpurun_out/art/bench.log; tail -2 gpurun_out/art/bench.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/art/prof -o run -- python3 bench.py --no-stream --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/art/prof_bench.log 2>&1; rc=$?
echo "rocprof exit=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/art/prof_bench.log; exit $rc; }
tail -1 gpurun_out/art/prof_bench.log | cut -c1-300
bash scripts/pmc_traffic.sh || exit 1
bash scripts/gpu_timeline.sh > gpurun_out/art/timeline.log 2>&1; rc=$?
tail -12 gpurun_out/art/timeline.log; exit $rc
