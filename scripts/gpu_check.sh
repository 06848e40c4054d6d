#!/bin/bash
# GPU-box check: pytest -m gpu, then a short bench. Stops on GPU fault / abort / timeout.
set -u
mkdir -p gpurun_out
TAG=${1:-run}
if [ "${SKIP_PYTEST:-0}" = "1" ]; then
  echo "pytest skipped" > gpurun_out/pytest_$TAG.log; rc=0
else
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -q -m gpu -rf --timeout 600 ${PYTEST_ARGS:-} > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
fi
echo "pytest exit=$rc" >> gpurun_out/pytest_$TAG.log
tail -15 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench_$TAG.log 2>&1
brc=$?
echo "bench exit=$brc" >> gpurun_out/bench_$TAG.log
tail -5 gpurun_out/bench_$TAG.log
if [ $brc -ne 0 ]; then exit $brc; fi
if [ "${CONVPROF:-1}" = "1" ]; then
  timeout -k 10 300 python scripts/conv_profile.py > gpurun_out/convprof_$TAG.log 2>&1
  crc=$?
  head -25 gpurun_out/convprof_$TAG.log
  if [ $crc -ne 0 ]; then echo "conv_profile exit=$crc"; exit $crc; fi
fi
if [ "${PROFILE:-0}" != "1" ]; then exit 0; fi
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG/bench.log 2>&1
prc=$?
echo "profile exit=$prc"
exit $prc
