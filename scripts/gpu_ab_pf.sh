#!/bin/bash
# A/B of the K = 1 L2 weight prefetch + 4-deep ring (RVC_X6_LD4_K=3) against the 2-deep ring (0)
set -u
O=gpurun_out/${TAG:-abpf}; mkdir -p $O
E="RVC_X6_LD4_K=0;RVC_X6_LD4_K=3;RVC_X6_LD4_K=0,RVC_SPLITK_TILES=0;RVC_X6_LD4_K=3,RVC_SPLITK_TILES=0"
timeout -k 10 300 python -u scripts/gemm_bench.py --precisions fp32 --envs "$E" > $O/gemm.log 2>&1; rc=$?
grep -v amdgpu.ids $O/gemm.log; exit $rc
