#!/bin/bash
# What bounds the K = 1 GEMM on the x6 engine: the ablation build (RVC_CONV_DEBUG 1 = no epilogue, 2 = no MFMA,
# 4 = loaders skip global loads; wrong results by design) on ContentVec's 2304 x 768 x 1599, split-K off
set -u
O=gpurun_out/${TAG:-ablg}; mkdir -p $O
L=$PWD/rvc-maker_amd/lib/abl/librvc_amd.so
E="RVC_SPLITK_TILES=0;RVC_SPLITK_TILES=0,RVC_CONV_DEBUG=1;RVC_SPLITK_TILES=0,RVC_CONV_DEBUG=2;RVC_SPLITK_TILES=0,RVC_CONV_DEBUG=4;RVC_SPLITK_TILES=0,RVC_CONV_DEBUG=6;RVC_SPLITK_TILES=0,RVC_CONV_DEBUG=7"
RVC_AMD_LIB=$L timeout -k 10 300 python -u scripts/gemm_bench.py --precisions fp32 --only 2,0 --envs "$E" > $O/abl.log 2>&1; rc=$?
grep -v amdgpu.ids $O/abl.log; exit $rc
