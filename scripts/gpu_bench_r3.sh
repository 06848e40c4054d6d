#!/bin/bash
# The default bench line, rocprofv3 kernel stats of the per-call bench, then the K = 1 GEMM A/B.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3b}; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1; rc=$?
tail -1 $O/bench.log | cut -c1-900; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-stream --steps 4 --warmup 1 --no-cpu-baseline > $O/prof_bench.log 2>&1; rc=$?
echo "rocprof exit=$rc"; tail -1 $O/prof_bench.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/gemm_bench.py > $O/gemm.log 2>&1; rc=$?
cat $O/gemm.log; exit $rc
