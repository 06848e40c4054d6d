#!/bin/bash
# round 5: f64 RMVPE buffers written by their producers (no zero fills) -- parity; epilogue issue-vs-retire stamps
set -o pipefail
O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rmvpe.py tests/test_gpu_ops.py -k "rmvpe or conv64 or wino or f64 or mel" > $O/t_rmvpe.log 2>&1 || { tail -30 $O/t_rmvpe.log; exit 1; }
tail -3 $O/t_rmvpe.log
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --only 0,1,3 --amax > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -v -i warn $O/stamps.log | grep -v amdgpu.ids
