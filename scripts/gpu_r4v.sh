#!/bin/bash
# 128-channel fused ResBlock pair: bit-identity / f16x3 tests, synth / pipeline tests, clip stream A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resblock.py > $O/t_rb.log 2>&1 || { tail -40 $O/t_rb.log; exit 1; }
tail -1 $O/t_rb.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_synth.py tests/test_gpu_native.py tests/test_gpu_pipeline.py > $O/t_syn.log 2>&1 || { tail -40 $O/t_syn.log; exit 1; }
tail -1 $O/t_syn.log
TAG=r4v/ab R=2 VARIANTS="rb128:RVC_X=1 off:RVC_AMD_FUSED_RB128=0" ./scripts/gpu_ab_env.sh
