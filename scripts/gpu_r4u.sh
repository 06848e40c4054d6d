#!/bin/bash
# occupancy-aware split-K target for the 8-compute-wave x6 tiles: GEMM shapes, conv suite tests, clip stream A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4u; mkdir -p $O
for v in 1 0; do RVC_X6_SPLIT_OCC=$v timeout -k 10 200 python -u scripts/gemm_bench.py > $O/gemm_$v.log 2>&1 || { tail $O/gemm_$v.log; exit 1; }; echo "occ=$v"; head -6 $O/gemm_$v.log | grep -v amdgpu; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_resblock.py tests/test_gpu_contentvec.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
TAG=r4u/ab R=2 VARIANTS="occ:RVC_X=1 old:RVC_X6_SPLIT_OCC=0" ./scripts/gpu_ab_env.sh
