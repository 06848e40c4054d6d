#!/bin/bash
# round 5: the x6 ping-pong form -- bit identity tests, per-shape timing, bench A/B
set -o pipefail
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "pingpong" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u scripts/pp_bench.py > $O/pp.log 2>&1 || { tail -20 $O/pp.log; exit 1; }
grep -v -i warn $O/pp.log | grep -v amdgpu.ids
for r in 1 2; do
for f in 0 1; do
RVC_X6_PP=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${f}_${r}.log 2>&1 || { tail -20 $O/b_${f}_${r}.log; exit 1; }
echo "pp=$f $(tail -1 $O/b_${f}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
