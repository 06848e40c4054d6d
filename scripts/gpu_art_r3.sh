#!/bin/bash
# Round-3 artifacts: the default bench line (CPU baseline + roofline), rocprofv3 kernel stats of the per-call
# bench (the roofline probe's setting), PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes), clip-stream timeline.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-art3}; mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1; rc=$?
tail -1 $O/bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-stream --steps 4 --warmup 1 --no-cpu-baseline > $O/prof_bench.log 2>&1; rc=$?
echo "rocprof exit=$rc"; tail -1 $O/prof_bench.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
if [ -z "${NO_PMC:-}" ]; then bash scripts/pmc_traffic.sh || exit 1
cp gpurun_out/pmc_traffic/summary.json $O/pmc_traffic.json; fi
[ -n "${NO_TL:-}" ] && exit 0
bash scripts/gpu_timeline.sh > $O/timeline.log 2>&1; rc=$?
cp gpurun_out/tl/timeline.txt $O/timeline.txt 2>/dev/null; tail -3 $O/timeline.log; exit $rc
