#!/bin/bash
# full GPU suite (one process), then smoke
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/full_test.log 2>&1; rc=$?
tail -8 gpurun_out/full_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -2 gpurun_out/smoke.log; exit $rc
