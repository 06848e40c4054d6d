#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_ivf.py tests/test_gpu_embedder_st.py tests/test_gpu_convert.py tests/test_gpu_bench.py > gpurun_out/r5a/tests.log 2>&1 || { tail -30 gpurun_out/r5a/tests.log; exit 1; }
tail -3 gpurun_out/r5a/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r5a/bench.log 2>&1 || { tail -20 gpurun_out/r5a/bench.log; exit 1; }
tail -c 1500 gpurun_out/r5a/bench.log
