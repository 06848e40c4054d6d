#!/bin/bash
# round 5: sharded |max| cells -- synth parity (both hosts) then interleaved A/B of the amax switches
set -o pipefail
O=gpurun_out/r5d; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_synth.py tests/test_gpu_native.py tests/test_gpu_ops.py -k "synth or native or conv or tile" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
for v in "0 1" "1 1" "1 0"; do set -- $v
RVC_AMD_AMAX=$1 RVC_AMD_AMAX_F16ALL=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/bench_$1$2_$r.log 2>&1 || { tail -20 $O/bench_$1$2_$r.log; exit 1; }
echo "amax=$1 f16all=$2 $(tail -1 $O/bench_$1$2_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
