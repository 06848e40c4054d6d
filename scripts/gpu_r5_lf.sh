#!/bin/bash
# round 5: fast-only split-fp16 loader kernels (LF) -- bit identity, stamps, bench A/B; RMVPE kernel trace
set -o pipefail
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "f16_fast or tile_epilogue or amax" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for f in 0 1; do
RVC_X6_F16FAST=$f RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,5,6 --amax > $O/stamps_$f.log 2>&1 || { tail -20 $O/stamps_$f.log; exit 1; }
echo "== f16fast $f"; grep -v -i warn $O/stamps_$f.log | grep -v amdgpu.ids | grep -v "CU period"
done
for r in 1 2; do
for f in 0 1; do
RVC_X6_F16FAST=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${f}_${r}.log 2>&1 || { tail -20 $O/b_${f}_${r}.log; exit 1; }
echo "f16fast=$f $(tail -1 $O/b_${f}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for pr in f64 fp32sa; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rm_$pr -o run -- python3 scripts/rmvpe_prof.py $pr 3 > $O/rm_$pr.log 2>&1 || { tail -20 $O/rm_$pr.log; exit 1; }
tail -1 $O/rm_$pr.log
done
