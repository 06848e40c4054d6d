#!/bin/bash
set -u
O=gpurun_out/r3i; mkdir -p $O
timeout -k 10 300 python -u scripts/dbg_native_index.py > $O/dbg.log 2>&1; tail -12 $O/dbg.log
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread -rf tests/test_gpu_ivf.py tests/test_gpu_native.py > $O/pytest.log 2>&1; rc=$?
tail -12 $O/pytest.log; exit $rc
