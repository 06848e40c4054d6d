#!/bin/bash
# One GPU-box session: steps named on the command line run in order, each under its own time limit;
# the session stops at the first failing step (no GPU step after a fault, abort or timeout).
#   bash scripts/gpu_run.sh TAG pytest bench bench2 cfg3 cfg5 prof
# PYTEST_ARGS narrows the pytest step (default: the whole -m gpu suite).
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc" >> "$OUT/$name.log"
  tail -4 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
for s in "$@"; do
  case $s in
    pytest) step pytest 1100 python -u -m pytest tests -q -m gpu --maxfail=${MAXFAIL:-1} -rf --timeout 900 --timeout-method thread ${PYTEST_ARGS:-} ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 2 ;;
    bench2) step bench2 600 python bench.py --gpus 2 --steps 5 --warmup 2 ;;
    graph) step graph 600 python bench.py --steps 10 --warmup 2 --graph --no-cpu-baseline ;;
    cfg3) step cfg3 600 python bench.py --steps 2 --warmup 1 --chunks 64 --seconds 10 --precision bf16x3 --index-rate 0.75 --no-cpu-baseline ;;
    cfg3b) step cfg3b 600 python bench.py --steps 2 --warmup 1 --chunks 64 --seconds 10 --precision bf16 --index-rate 0.75 --no-cpu-baseline ;;
    cfg5) step cfg5 600 python bench.py --steps 2 --warmup 1 --chunks 4 --sr 40000 --f0 crepe-full --precision bf16x3 --graph --no-cpu-baseline ;;
    micro) step micro 300 python scripts/micro.py branches ;;
    convprof) step convprof 300 python scripts/conv_profile.py ;;
    prof)
      export TMPDIR=/tmp
      step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all steps ok"
