#!/bin/bash
# Round-4 end-of-round numbers for the BASELINE config variants (one MI355X).
set -o pipefail
O=gpurun_out/r4cfg; mkdir -p $O
timeout -k 10 500 python -u bench.py --no-cpu-baseline --chunks 64 --seconds 10 --index-rate 0.75 --precision bf16x3 --batch 8 > $O/cfg3.log 2>&1 && \
timeout -k 10 500 python -u bench.py --no-cpu-baseline --sr 40000 --f0 crepe-full --precision bf16x3 --graph --chunks 4 > $O/cfg5.log 2>&1 && \
timeout -k 10 500 python -u bench.py --no-cpu-baseline --precision bf16x3 > $O/cfg1_bf16x3.log 2>&1
rc=$?
for f in cfg3 cfg5 cfg1_bf16x3; do grep '"metric"' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d.get('per_call'), json.dumps(d['config']))"; done
exit $rc
