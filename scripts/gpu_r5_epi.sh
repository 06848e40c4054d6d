#!/bin/bash
# round 5: the x6 tile epilogue -- bit-identity and conv unit tests, the pipeline goldens, stamps, conv A/B, bench
set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_resblock.py tests/test_gpu_pipeline.py tests/test_gpu_synth.py tests/test_gpu_batch.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --out $O/stamps_fp32.json > $O/stamps_fp32.log 2>&1 || { tail -20 $O/stamps_fp32.log; exit 1; }
grep -v Warn $O/stamps_fp32.log | grep -v warn
for v in 0 1 0 1; do RVC_X6_TILE_EPI=$v timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 > $O/cb_$v.log 2>&1 || { tail -20 $O/cb_$v.log; exit 1; }; echo "tile_epi=$v"; cat $O/cb_$v.log; done
for v in 1 0 1; do RVC_X6_TILE_EPI=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }; echo "tile_epi=$v $(tail -1 $O/bench_$v.log | cut -c1-300)"; done
