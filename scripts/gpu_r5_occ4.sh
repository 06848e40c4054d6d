#!/bin/bash
# round 5: the 64 x 128 split-fp16 tile at 4 waves per SIMD (two 8-wave blocks per CU) -- tests with it on, conv
# timings, bench A/B; then the end-of-round conv precision table and stamps
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O
export RVC_AMD_LIB=rvc-maker_amd/lib/o/librvc_amd.so
RVC_X6_OCC4=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_synth.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for o in 0 1; do
RVC_X6_OCC4=$o timeout -k 10 300 python -u scripts/conv_bench.py --precision f16x3 --reps 5 > $O/cb_$o.log 2>&1 || { tail -20 $O/cb_$o.log; exit 1; }
echo "== occ4 $o"; grep -v -i warn $O/cb_$o.log | grep -v amdgpu.ids
done
for r in 1 2; do
for o in 0 1; do
RVC_X6_OCC4=$o timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${o}_${r}.log 2>&1 || { tail -20 $O/b_${o}_${r}.log; exit 1; }
echo "occ4=$o $(tail -1 $O/b_${o}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
unset RVC_AMD_LIB
timeout -k 10 300 python -u scripts/conv_prec.py --gen --out $O/conv_prec_gen.txt > $O/conv_prec.log 2>&1 || { tail -20 $O/conv_prec.log; exit 1; }
cat $O/conv_prec_gen.txt
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --amax --only 0,1,2,6,7,8,9 --out $O/conv_stamps.json > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -v -i warn $O/stamps.log | grep -v amdgpu.ids | head -40
