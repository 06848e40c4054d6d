#!/bin/bash
# Round-4 final artifacts (final tree): full -m gpu suite, smoke, rocprofv3 summary of the bench, PMC traffic
# stamped with the kernel-source hash, then the default bench line with the traffic filled in.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-final6}; mkdir -p $O
timeout -k 10 2400 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/gpu_suite.log 2>&1 || { tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 600 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep '"metric"' $O/prof.log | cut -c1-200
bash scripts/pmc_traffic.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cp gpurun_out/pmc_traffic/summary.json $O/pmc_traffic.json
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['per_call'], json.dumps(d['roofline'])[:400]); print(json.dumps(d['cpu_baseline'])[:300])"
