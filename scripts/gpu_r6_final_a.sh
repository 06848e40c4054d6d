#!/bin/bash
# round 6, end of round (1/2): the whole -m gpu suite, smoke, two default bench lines.
set -o pipefail
O=gpurun_out/r6final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?
tail -3 $O/suite.log
grep -E "^FAILED" $O/suite.log | head -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stop"; exit 1; fi
grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/suite.log && { echo "GPU fault: stop"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 400 python -u bench.py > $O/bench_$r.log 2>&1 || { tail -20 $O/bench_$r.log; exit 1; }
  grep '^{' $O/bench_$r.log | tail -1 | cut -c1-200
done
