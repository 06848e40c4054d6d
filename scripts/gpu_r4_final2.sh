#!/bin/bash
# PMC traffic passes (stamped with the kernel-source hash), then the default bench line with the traffic filled in.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-final7}; mkdir -p $O
bash scripts/pmc_traffic.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cp gpurun_out/pmc_traffic/summary.json $O/pmc_traffic.json
cp gpurun_out/pmc_traffic/summary.json profiles/r4_pmc_traffic.json
head -c 1500 $O/pmc_traffic.json; echo
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:600], d.get('per_call'))"
