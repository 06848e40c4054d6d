#!/bin/bash
# round 5: staggered first-round start of the x6 blocks -- stamps (epilogue under HBM contention) and bench A/B
set -o pipefail
O=gpurun_out/r5j; mkdir -p $O
for st in 0 30000 60000; do
RVC_X6_STAGGER=$st RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,2,3,5,6 --amax > $O/stamps_$st.log 2>&1 || { tail -20 $O/stamps_$st.log; exit 1; }
echo "== stagger $st"; grep -v -i warn $O/stamps_$st.log | grep -v amdgpu.ids
done
for r in 1 2; do
for st in 0 30000 60000; do
RVC_X6_STAGGER=$st timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${st}_${r}.log 2>&1 || { tail -20 $O/b_${st}_${r}.log; exit 1; }
echo "stagger=$st $(tail -1 $O/b_${st}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
