#!/bin/bash
# A/B of the x6 engine's XCD tile order and 4-deep input ring: ContentVec's K = 1 GEMMs and the generator shapes
set -u
O=gpurun_out/${TAG:-abx6}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_contentvec.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
E="RVC_X6_XCD=0,RVC_X6_LD4_K=0;RVC_X6_XCD=1,RVC_X6_LD4_K=0;RVC_X6_XCD=0,RVC_X6_LD4_K=3;RVC_X6_XCD=1,RVC_X6_LD4_K=3"
timeout -k 10 300 python -u scripts/gemm_bench.py --precisions fp32 --envs "$E" > $O/gemm.log 2>&1; rc=$?
cat $O/gemm.log; [ $rc -ne 0 ] && exit $rc
for x in 0 1; do
  echo "conv_bench RVC_X6_XCD=$x"
  RVC_X6_XCD=$x timeout -k 10 300 python -u scripts/conv_bench.py --reps 5 > $O/conv_xcd$x.log 2>&1 || exit $?
  tail -12 $O/conv_xcd$x.log
done
for x in 0 1; do
  RVC_X6_XCD=$x RVC_X6_LD4_K=$((3*x)) timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 10 --warmup 3 > $O/bench$x.log 2>&1 || exit $?
  echo "bench xcd/ld4 $x: $(grep -o '"value": [0-9.]*' $O/bench$x.log | head -2 | tr '\n' ' ')"
done
