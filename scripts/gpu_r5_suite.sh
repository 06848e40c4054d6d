#!/bin/bash
# round 5: the whole -m gpu suite, stamps of the cell-mode prologue (one barrier less), epilogue contention stamps,
# bench
set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,7,8 --amax > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -v -i warn $O/stamps.log | grep -v amdgpu.ids | grep -v "CU period"
bash scripts/gpu_r5_epi3.sh
for r in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_$r.log 2>&1 || { tail -20 $O/b_$r.log; exit 1; }
echo "bench $(tail -1 $O/b_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done
