#!/bin/bash
# Round-3 check on one box: the whole -m gpu suite, smoke, the default bench line, and the rocprofv3 kernel
# stats of the per-call bench (the roofline probe's setting).  Every GPU step has its own time limit; the
# script stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1; rc=$?
tail -1 $O/bench.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-stream --steps 4 --warmup 1 --no-cpu-baseline > $O/prof_bench.log 2>&1; rc=$?
echo "rocprof exit=$rc"; tail -1 $O/prof_bench.log | cut -c1-300
exit $rc
