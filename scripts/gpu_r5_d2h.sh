#!/bin/bash
# round 5: D2H on the back stream (front end free to run ahead); amax / fast-F16 A/B; stamps; timeline
set -o pipefail
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench.py tests/test_gpu_ops.py -k "bench or fe0 or tile" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
for v in "1 1 0" "0 1 0" "1 0 0" "1 1 1"; do set -- $v
h=""; [ $3 = 1 ] && h="--hbm-output"
RVC_AMD_AMAX=$1 RVC_X6_F16FAST=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 $h > $O/bench_$1$2$3_$r.log 2>&1 || { tail -20 $O/bench_$1$2$3_$r.log; exit 1; }
echo "amax=$1 f16fast=$2 hbm_out=$3 $(tail -1 $O/bench_$1$2$3_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
RVC_X6_F16FAST=0 RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,2,3 --amax --out $O/stamps_amax_nofast.json > $O/stamps_amax_nofast.log 2>&1 || { tail -20 $O/stamps_amax_nofast.log; exit 1; }
echo "== stamps amax, general loader"; grep -v -i warn $O/stamps_amax_nofast.log | grep -v amdgpu.ids
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-per-call --no-roofline > $O/tl_bench.log 2>&1 || { tail -20 $O/tl_bench.log; exit 1; }
f=$(find $O/tl -name "*kernel_trace.csv" | head -1)
python scripts/timeline.py "$f" > $O/timeline.txt 2>&1; head -8 $O/timeline.txt
gzip -f "$f"
