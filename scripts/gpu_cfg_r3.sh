#!/bin/bash
# Clip-stream timeline under rocprofv3 (masked synthesizer stream), then BASELINE cfg 3 / cfg 5 bench variants
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-cfg3r}; mkdir -p $O
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-roofline --chunks 64 --seconds 10 --index-rate 0.75 --precision bf16x3 --batch 8 --steps 2 --warmup 1 > $O/cfg3.log 2>&1 || { tail -3 $O/cfg3.log; exit 1; }
echo "cfg3 $(grep -o '"value": [0-9.]*' $O/cfg3.log | head -2 | tr '\n' ' ')"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-roofline --sr 40000 --f0 crepe-full --precision bf16x3 --graph --chunks 4 --steps 3 --warmup 1 > $O/cfg5.log 2>&1 || { tail -3 $O/cfg5.log; exit 1; }
echo "cfg5 $(grep -o '"value": [0-9.]*' $O/cfg5.log | head -1)"
bash scripts/gpu_timeline.sh > $O/timeline.log 2>&1; rc=$?
cp gpurun_out/tl/timeline.txt $O/timeline.txt 2>/dev/null; tail -4 $O/timeline.log | cut -c1-200; exit $rc
