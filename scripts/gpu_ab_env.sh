#!/bin/bash
# Interleaved bench A/B of environment settings on one box: VARIANTS="name:ENV=V,ENV2=V2 name2:..." (rounds R)
set -u
O=gpurun_out/${TAG:-abenv}; mkdir -p $O
for r in $(seq 1 ${R:-2}); do
  for v in $VARIANTS; do
    name=${v%%:*}; envs=${v#*:}
    env $(echo $envs | tr ',' ' ') timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --no-per-call --steps ${STEPS:-12} --warmup 3 ${BENCH_ARGS:-} > $O/${name}_$r.log 2>&1 || { tail -3 $O/${name}_$r.log; exit 1; }
    echo "$name#$r $(grep -o '"value": [0-9.]*' $O/${name}_$r.log | head -1)"
  done
done
