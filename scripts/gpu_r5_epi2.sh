#!/bin/bash
# round 5: the x6 epilogue's cost against tile width and the number of CUs storing at once (stamps)
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
for bn in 3 0; do
RVC_X6_BN256=$bn RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,1,2,3,5 --amax > $O/stamps_bn$bn.log 2>&1 || { tail -20 $O/stamps_bn$bn.log; exit 1; }
echo "== bn256 $bn"; grep -v -i warn $O/stamps_bn$bn.log | grep -v amdgpu.ids
done
