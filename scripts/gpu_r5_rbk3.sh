#!/bin/bash
# round 5: the fused ResBlock pairs at K = 3 in split-fp16 (RVC_AMD_RB_F16_KMIN=3) -- pair timings, bench A/B
set -o pipefail
O=gpurun_out/r5z; mkdir -p $O
for k in 7 3; do
RVC_AMD_RB_F16_KMIN=$k timeout -k 10 300 python -u scripts/rb_bench.py > $O/rb_$k.log 2>&1 || { tail -20 $O/rb_$k.log; exit 1; }
echo "== kmin $k"; grep -v -i warn $O/rb_$k.log | grep -v amdgpu.ids | tail -12
done
for r in 1 2; do
for k in 7 3; do
RVC_AMD_RB_F16_KMIN=$k timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${k}_${r}.log 2>&1 || { tail -20 $O/b_${k}_${r}.log; exit 1; }
echo "kmin=$k $(tail -1 $O/b_${k}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
