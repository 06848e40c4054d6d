#!/bin/bash
# GPU-box check: pytest -m gpu, then a short bench. Stops on GPU fault / abort / timeout.
set -u
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -q -m gpu -rf --timeout 600 ${PYTEST_ARGS:-} > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/pytest_$TAG.log
tail -15 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench_$TAG.log 2>&1
brc=$?
echo "bench exit=$brc" >> gpurun_out/bench_$TAG.log
tail -5 gpurun_out/bench_$TAG.log
exit $brc
