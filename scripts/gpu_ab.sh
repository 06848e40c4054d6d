#!/bin/bash
# Conv-engine A/B on the GPU box: conv_bench (with --check) per env setting; usage: gpu_ab.sh "ENV1" "ENV2" ...
set -u
mkdir -p gpurun_out
PREC=${PREC:-fp32}
i=0
for e in "$@"; do
  i=$((i+1))
  echo "== [$e] precision $PREC"
  env $e timeout -k 10 120 python -u scripts/conv_bench.py --reps 5 --check --precision $PREC ${CB_ARGS:-} > gpurun_out/ab_$i.log 2>&1
  rc=$?
  grep -E "C=|total|Error|error" gpurun_out/ab_$i.log | cut -c1-150
  if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi
done
