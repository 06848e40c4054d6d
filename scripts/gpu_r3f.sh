#!/bin/bash
set -u
O=gpurun_out/r3f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 250 --timeout-method thread -rf tests/test_gpu_ops.py > $O/ops.log 2>&1; rc=$?
tail -5 $O/ops.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/conv_prec.py > $O/conv_prec.log 2>&1 || { tail -20 $O/conv_prec.log; exit 1; }
cat $O/conv_prec.log
timeout -k 10 300 python -u scripts/rmvpe_prec.py 30 201 > $O/prec.log 2>&1 || { tail -20 $O/prec.log; exit 1; }
tail -13 $O/prec.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-1500
