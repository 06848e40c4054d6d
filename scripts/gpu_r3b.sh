#!/bin/bash
# RMVPE precision after the f64 STFT, then the RMVPE-dependent parity tests
set -u
mkdir -p gpurun_out/r3d
timeout -k 10 300 python -u scripts/rmvpe_prec.py 30 201 > gpurun_out/r3d/prec.log 2>&1 || { tail -20 gpurun_out/r3d/prec.log; exit 1; }
tail -14 gpurun_out/r3d/prec.log
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread -rf tests/test_gpu_rmvpe.py tests/test_gpu_pipeline.py tests/test_gpu_native.py tests/test_gpu_batch.py "tests/test_gpu_configs.py::test_cfg2_headline_30s_48k_fp32_vs_oracle" > gpurun_out/r3d/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r3d/pytest.log; cp gpurun_out/config_parity.json gpurun_out/r3d/ 2>/dev/null; exit $rc
