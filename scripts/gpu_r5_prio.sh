#!/bin/bash
# round 5: stream priorities A/B (the f64 RMVPE chain waits for CUs behind the high-priority synthesizer stream)
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O
for r in 1 2; do
for v in "0 0 -1" "-1 0 -1" "-1 -1 -1" "-1 -1 0" "-1 0 0"; do set -- $v
RVC_AMD_FSIDE_PRIORITY=$1 RVC_AMD_FRONT_PRIORITY=$2 RVC_AMD_BACK_PRIORITY=$3 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_$r.log 2>&1 || { tail -20 $O/b_$r.log; exit 1; }
echo "fside=$1 front=$2 back=$3 $(tail -1 $O/b_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,2,3 --amax > $O/stamps_amax.log 2>&1 || { tail -20 $O/stamps_amax.log; exit 1; }
grep -v -i warn $O/stamps_amax.log | grep -v amdgpu.ids
