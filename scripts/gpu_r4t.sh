#!/bin/bash
# K = 1 GEMMs on the f32 MFMA engine vs the split-bf16 engine: gemm_bench shapes and the clip stream.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4t; mkdir -p $O
for k1 in 1 0; do RVC_X6_K1=$k1 timeout -k 10 200 python -u scripts/gemm_bench.py > $O/gemm_k1_$k1.log 2>&1 || { tail $O/gemm_k1_$k1.log; exit 1; }; echo "k1=$k1"; tail -8 $O/gemm_k1_$k1.log; done
TAG=r4t/ab R=2 VARIANTS="x6:RVC_X=1 f32k1:RVC_X6_K1=0" ./scripts/gpu_ab_env.sh
