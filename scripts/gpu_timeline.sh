#!/bin/bash
# rocprofv3 kernel trace of the clip-stream bench; stream timeline summary.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 bench.py --steps ${STEPS:-6} --warmup 1 --no-cpu-baseline --no-per-call --no-roofline ${MODE:-} > gpurun_out/tl/bench.log 2>&1
rc=$?
echo "profile exit=$rc"; tail -1 gpurun_out/tl/bench.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1)
head -1 "$f"
python scripts/timeline.py "$f" > gpurun_out/tl/timeline.txt 2>&1; cat gpurun_out/tl/timeline.txt
gzip -f "$f"
