#!/bin/bash
# round 5: the amax cell read through the scalar cache -- stamps with / without, bench A/B
set -o pipefail
O=gpurun_out/r5h; mkdir -p $O
for a in "" "--amax"; do
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,2,3 $a > $O/stamps$a.log 2>&1 || { tail -20 $O/stamps$a.log; exit 1; }
echo "== stamps $a"; grep -v -i warn $O/stamps$a.log | grep -v amdgpu.ids
done
for r in 1 2; do
for v in 1 0; do
RVC_AMD_AMAX=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${v}_${r}.log 2>&1 || { tail -20 $O/b_${v}_${r}.log; exit 1; }
echo "amax=$v $(tail -1 $O/b_${v}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
for r in 1 2; do
for v in "1 4" "2 8" "3 12"; do set -- $v
RVC_STREAM_FRONTS=$1 GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --no-per-call --steps 12 --warmup 3 > $O/f_$1_$r.log 2>&1 || { tail -20 $O/f_$1_$r.log; exit 1; }
echo "fronts=$1 queues=$2 $(tail -1 $O/f_$1_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done; done
