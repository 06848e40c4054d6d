#!/bin/bash
# rocprofv3 HIP API + kernel trace of the clip-stream bench: which host calls block inside the stream.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ht
timeout -k 10 600 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/ht -o run -- python3 bench.py --steps ${STEPS:-6} --warmup 1 --no-cpu-baseline --no-per-call --no-roofline ${MODE:-} > gpurun_out/ht/bench.log 2>&1
rc=$?
echo "profile exit=$rc"; tail -1 gpurun_out/ht/bench.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
for f in $(find gpurun_out/ht -name "*_trace.csv"); do head -1 $f; gzip -f $f; done
ls -la gpurun_out/ht
