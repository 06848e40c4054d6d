#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run; usage: gpu_prof.sh TAG [bench args]
set -u
TAG=${1:?tag}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG/bench.log 2>&1
rc=$?
echo "profile exit=$rc"
tail -1 gpurun_out/prof_$TAG/bench.log | cut -c1-200
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -3
exit $rc
