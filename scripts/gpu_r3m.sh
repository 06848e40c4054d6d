#!/bin/bash
# perf A/B: split-K target grid on the headline stream; cfg 3 (64 x 10 s, batch 8, index 0.75, bf16x3) with the
# batched synthesizer on / off
set -u
O=gpurun_out/${TAG:-r3m}; mkdir -p $O
B="python -u bench.py --no-cpu-baseline --no-per-call --no-roofline"
for t in 512 256 128 0; do
  RVC_SPLITK_TILES=$t timeout -k 10 300 $B --steps 10 --warmup 3 > $O/head_splitk$t.log 2>&1 || exit $?
  echo "splitk $t: $(grep -o '"value": [0-9.]*' $O/head_splitk$t.log)"
done
for sb in 1 0; do
  RVC_AMD_SYNTH_BATCH=$sb timeout -k 10 400 $B --chunks 64 --batch 8 --seconds 10 --index-rate 0.75 \
    --precision bf16x3 --steps 2 --warmup 1 > $O/cfg3_sb$sb.log 2>&1 || exit $?
  echo "cfg3 synth_batch $sb: $(grep -o '"value": [0-9.]*' $O/cfg3_sb$sb.log)"
done
bash scripts/gpu_prof.sh ${TAG:-r3m}_head --no-per-call --no-roofline || exit $?
