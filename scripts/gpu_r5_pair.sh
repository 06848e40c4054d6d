#!/bin/bash
# round 5: the paired x6 form (128 x 128 tiles, 4 compute + 2 loader waves, 2 blocks per CU) -- tests with it on,
# stamps, bench A/B
set -o pipefail
O=gpurun_out/r5t; mkdir -p $O
RVC_X6_PAIR=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_synth.py tests/test_gpu_resblock.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for pr in 0 1; do
RVC_X6_PAIR=$pr RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,6,7,8,9 --amax > $O/stamps_$pr.log 2>&1 || { tail -20 $O/stamps_$pr.log; exit 1; }
echo "== pair $pr"; grep -v -i warn $O/stamps_$pr.log | grep -v amdgpu.ids | grep -v "CU period"
done
for r in 1 2; do
for pr in 0 1; do
RVC_X6_PAIR=$pr timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${pr}_${r}.log 2>&1 || { tail -20 $O/b_${pr}_${r}.log; exit 1; }
echo "pair=$pr $(tail -1 $O/b_${pr}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
