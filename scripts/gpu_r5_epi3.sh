#!/bin/bash
# round 5: is the x6 epilogue bound by chip-wide contention? one round of 256-wide blocks on 64..256 CUs, and the
# 256-CU round with its starts spread (stagger) -- stamps
set -o pipefail
O=gpurun_out/r5q; mkdir -p $O
for st in 0 150000; do
RVC_X6_BN256=3 RVC_X6_STAGGER=$st RVC_X6_STAGGER_ROUNDS=1 RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 2,3,4,5 --amax > $O/stamps_$st.log 2>&1 || { tail -20 $O/stamps_$st.log; exit 1; }
echo "== stagger $st"; grep -v -i warn $O/stamps_$st.log | grep -v amdgpu.ids | grep -v "per chunk"
done
