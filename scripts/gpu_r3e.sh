#!/bin/bash
set -u
O=gpurun_out/r3e; mkdir -p $O
timeout -k 10 300 python -u scripts/conv_prec.py > $O/conv_prec.log 2>&1 || { tail -20 $O/conv_prec.log; exit 1; }
cat $O/conv_prec.log
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread -rf tests/test_gpu_rmvpe.py tests/test_gpu_native.py tests/test_gpu_ivf.py tests/test_gpu_pipeline.py "tests/test_gpu_configs.py::test_cfg2_headline_30s_48k_fp32_vs_oracle" "tests/test_gpu_configs.py::test_cfg3_index_chunks_vs_oracle" > $O/pytest.log 2>&1; rc=$?
tail -25 $O/pytest.log; cp gpurun_out/config_parity.json $O/ 2>/dev/null; exit $rc
