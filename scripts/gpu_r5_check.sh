#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_ivf.py tests/test_gpu_embedder_st.py tests/test_gpu_convert.py tests/test_gpu_bench.py > gpurun_out/r5a/tests.log 2>&1 || { tail -30 gpurun_out/r5a/tests.log; exit 1; }
tail -3 gpurun_out/r5a/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r5a/bench.log 2>&1 || { tail -20 gpurun_out/r5a/bench.log; exit 1; }
tail -c 1500 gpurun_out/r5a/bench.log
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --out gpurun_out/r5a/stamps_fp32.json > gpurun_out/r5a/stamps_fp32.log 2>&1 || { tail -20 gpurun_out/r5a/stamps_fp32.log; exit 1; }
cat gpurun_out/r5a/stamps_fp32.log
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --precision f16x3 --out gpurun_out/r5a/stamps_f16.json > gpurun_out/r5a/stamps_f16.log 2>&1 || { tail -20 gpurun_out/r5a/stamps_f16.log; exit 1; }
cat gpurun_out/r5a/stamps_f16.log
