#!/bin/bash
# round 5: the loaders' epilogue prefetch (LDS-DMA of the residual / accumulate rows during the last chunk) --
# conv tests, stamps, bench A/B
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_resblock.py tests/test_gpu_synth.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for pf in 0 1; do
RVC_X6_EPI_PF=$pf RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,7,8 --amax > $O/stamps_$pf.log 2>&1 || { tail -20 $O/stamps_$pf.log; exit 1; }
echo "== epi_pf $pf"; grep -v -i warn $O/stamps_$pf.log | grep -v amdgpu.ids | grep -v "CU period" | grep -v "per chunk"
done
for r in 1 2; do
for pf in 0 1; do
RVC_X6_EPI_PF=$pf timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${pf}_${r}.log 2>&1 || { tail -20 $O/b_${pf}_${r}.log; exit 1; }
echo "epi_pf=$pf $(tail -1 $O/b_${pf}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
