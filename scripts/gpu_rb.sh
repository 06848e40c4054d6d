#!/bin/bash
# fused ResBlock session: its tests, the synthesizer / pipeline goldens, then bench A/B (fused vs two-launch) and the conv profile
set -u
OUT=gpurun_out/rb; mkdir -p $OUT
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -3 $OUT/$name.log | cut -c1-300; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
run t_rb 300 python -u -m pytest tests/test_gpu_resblock.py -x -q --timeout 200 --timeout-method thread
run t_synth 400 python -u -m pytest tests/test_gpu_synth.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread
run bench_fused 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
RVC_AMD_FUSED_RB=0 run bench_unfused 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
run convprof 300 python scripts/conv_profile.py --top 40
echo all ok
