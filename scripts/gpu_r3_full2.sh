#!/bin/bash
# Whole -m gpu suite, then micro-benches and the default bench line
set -u
O=gpurun_out/${TAG:-r3f2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/gemm_bench.py --precisions fp32 --envs "RVC_X6_XCD=1" > $O/gemm.log 2>&1 || exit 1
grep total $O/gemm.log
timeout -k 10 200 python -u scripts/conv_bench.py --reps 5 > $O/conv.log 2>&1 || exit 1
tail -1 $O/conv.log
timeout -k 10 200 python -u scripts/rb_bench.py --reps 5 > $O/rb.log 2>&1 || exit 1
tail -1 $O/rb.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-300
