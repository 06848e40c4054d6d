#!/bin/bash
# round 5, end of round (after the ContentVec |max| cells): the whole -m gpu suite, smoke, default bench lines,
# rocprofv3 kernel stats of the bench, PMC traffic on this tree, RMVPE alone under rocprofv3
set -o pipefail
O=gpurun_out/r5final2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
timeout -k 10 400 python -u bench.py > $O/bench_$r.log 2>&1 || { tail -20 $O/bench_$r.log; exit 1; }
tail -1 $O/bench_$r.log | cut -c1-300
done
bash scripts/gpu_prof.sh r5b || exit 1
bash scripts/pmc_traffic.sh > $O/pmc_traffic.log 2>&1 || { tail -20 $O/pmc_traffic.log; exit 1; }
tail -8 $O/pmc_traffic.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rm -o run -- python3 scripts/rmvpe_prof.py f64 3 > $O/rm.log 2>&1 || { tail -20 $O/rm.log; exit 1; }
grep "RMVPE" $O/rm.log
