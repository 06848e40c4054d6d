#!/bin/bash
# round 5: fused ContentVec layer 0 parity; conv stamps with / without the producer's |max|; stream timeline; bench
set -o pipefail
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_contentvec.py tests/test_gpu_native.py tests/test_gpu_batch.py tests/test_gpu_pipeline.py tests/test_gpu_embedder_st.py tests/test_gpu_extract.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for a in "" "--amax"; do
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,1,2,3,4 $a --out $O/stamps$a.json > $O/stamps$a.log 2>&1 || { tail -20 $O/stamps$a.log; exit 1; }
echo "== stamps $a"; grep -v -i warn $O/stamps$a.log | grep -v amdgpu.ids
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-per-call --no-roofline > $O/tl_bench.log 2>&1 || { tail -20 $O/tl_bench.log; exit 1; }
f=$(find $O/tl -name "*kernel_trace.csv" | head -1)
python scripts/timeline.py "$f" > $O/timeline.txt 2>&1; cat $O/timeline.txt | head -80
gzip -f "$f"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
