#!/bin/bash
# After the static-vmcnt prefetch rewrite: engine / ResBlock / ContentVec parity tests, then the micro-benches and
# the default bench line
set -u
O=gpurun_out/${TAG:-r3s}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_resblock.py tests/test_gpu_synth.py tests/test_gpu_contentvec.py tests/test_gpu_rmvpe.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/gemm_bench.py --precisions fp32 --envs "RVC_X6_LD4_K=0;RVC_X6_LD4_K=3" > $O/gemm.log 2>&1 || exit 1
grep -v amdgpu.ids $O/gemm.log
timeout -k 10 200 python -u scripts/conv_bench.py --reps 5 > $O/conv.log 2>&1 || exit 1
tail -10 $O/conv.log
timeout -k 10 200 python -u scripts/rb_bench.py --reps 5 > $O/rb.log 2>&1 || exit 1
tail -13 $O/rb.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-300
