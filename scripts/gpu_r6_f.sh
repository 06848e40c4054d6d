#!/bin/bash
# round 6, sixth GPU pass: block-level |max| publishing (split-K reduce over row blocks, source pass, LayerNorms,
# embedding, rel-v band), the wide C = 64 pair's batched epilogue loads; the touched suites, per-tile stamps of both
# C = 64 geometries, the synthesizer's stages per switch, an interleaved end-to-end A/B and a kernel summary.
set -o pipefail
O=gpurun_out/r6f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest --maxfail=20 -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_resblock.py tests/test_gpu_ops.py tests/test_gpu_amax.py tests/test_gpu_synth.py tests/test_gpu_native.py \
  tests/test_gpu_contentvec.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1
rc=$?
tail -30 $O/tests.log | grep -v "^\.\.\.\." | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stop"; exit 1; fi
grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/tests.log && { echo "GPU fault: stop"; exit 1; }
for w in 1 0; do
  RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 200 python -u scripts/rb_stamps.py --wide64 $w \
    --out $O/rb_stamps_w$w.json > $O/rb_stamps_w$w.log 2>&1 || { tail -5 $O/rb_stamps_w$w.log; exit 1; }
  grep -E "^c(32|64)" $O/rb_stamps_w$w.log | cut -c1-200
done
timeout -k 10 300 python -u scripts/synth_stage_time.py --out $O/synth_stages.json base ATTN_F16=0 TE_AMAX=1 FLOW_AMAX=1 \
  > $O/synth_stages.log 2>&1 || { tail -5 $O/synth_stages.log; exit 1; }
grep -v amdgpu.ids $O/synth_stages.log
TAG=r6f/ab VARIANTS="new:RVC_X=1 wide0:RVC_RB_WIDE64=0 te1:RVC_AMD_TE_AMAX=1 flow1:RVC_AMD_FLOW_AMAX=1 rb128:RVC_AMD_FUSED_RB128=1" R=2 bash scripts/gpu_ab_env.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-per-call > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1):8 > $O/kstats.txt 2>&1 || true
head -24 $O/kstats.txt
