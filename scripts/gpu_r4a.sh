#!/bin/bash
# Round 4 A/B: BiGRU64 microbench, conv correctness on the new loader, conv_bench old vs new, RMVPE f64 time,
# bench (new, then the HEAD build in lib/old for comparison).  Each GPU step under its own time limit; stops at
# the first failure.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r4a
mkdir -p $O
step() { local t=$1; shift; echo "== $*"; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
step 150 ./scripts/bigru64_bench 3232 > $O/bigru64_bench.log 2>&1; cat $O/bigru64_bench.log
step 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_resblock.py > $O/tests_ops.log 2>&1; tail -3 $O/tests_ops.log
step 200 python -u scripts/conv_bench.py --only 3,4,1 > $O/conv_new.log 2>&1; cat $O/conv_new.log
RVC_AMD_LIB=$PWD/rvc-maker_amd/lib/old/librvc_amd.so step 200 python -u scripts/conv_bench.py --only 3,4,1 > $O/conv_old.log 2>&1; cat $O/conv_old.log
step 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rmvpe_f64.log 2>&1; tail -1 $O/rmvpe_f64.log
step 300 python -u bench.py --no-cpu-baseline > $O/bench_new.log 2>&1; tail -1 $O/bench_new.log | cut -c1-300
RVC_AMD_LIB=$PWD/rvc-maker_amd/lib/old/librvc_amd.so step 300 python -u bench.py --no-cpu-baseline --no-roofline > $O/bench_old.log 2>&1; tail -1 $O/bench_old.log | cut -c1-300
step 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rmvpe.py tests/test_gpu_native.py tests/test_gpu_batch.py > $O/tests_rm.log 2>&1; tail -3 $O/tests_rm.log
