#!/bin/bash
# HBM traffic of the bench's conv kernels from PMC: one rocprofv3 pass per counter (FETCH_SIZE, then
# WRITE_SIZE; they cannot share a pass), over one eager bench step.  Summarised by pmc_traffic.py.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_traffic
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_traffic/$c -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream > gpurun_out/pmc_traffic/$c.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc $c rc=$rc"; tail -5 gpurun_out/pmc_traffic/$c.log; exit $rc; fi
done
python3 scripts/pmc_traffic.py gpurun_out/pmc_traffic > gpurun_out/pmc_traffic/summary.json && cat gpurun_out/pmc_traffic/summary.json
