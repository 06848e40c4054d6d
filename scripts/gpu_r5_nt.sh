#!/bin/bash
# round 5: non-temporal epilogue stores / residual loads (RVC_CONV_NT) -- stamps and bench A/B
set -o pipefail
O=gpurun_out/r5l; mkdir -p $O
for nt in 0 1 2 3; do
RVC_CONV_NT=$nt RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,1,5 --amax > $O/stamps_$nt.log 2>&1 || { tail -20 $O/stamps_$nt.log; exit 1; }
echo "== nt $nt"; grep -v -i warn $O/stamps_$nt.log | grep -v amdgpu.ids | grep -v "CU period"
done
for r in 1 2; do
for nt in 0 3 1; do
RVC_CONV_NT=$nt timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${nt}_${r}.log 2>&1 || { tail -20 $O/b_${nt}_${r}.log; exit 1; }
echo "nt=$nt $(tail -1 $O/b_${nt}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
