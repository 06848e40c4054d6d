#!/bin/bash
# round 5: the default bench line on the final tree, now that profiles/r5_pmc_traffic.json matches its source hash
set -o pipefail
O=gpurun_out/r5bl; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
