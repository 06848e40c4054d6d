#!/bin/bash
# round 6, second GPU pass: the source-conv pass out of the conv epilogue (the fused form had taken the 128 x 256 tile's
# spills 31 -> 154 VGPRs), the fused pair's outputs through LDS; the touched suites, a per-feature interleaved A/B
# (each round-6 default switched off alone, and all of them), the pair stamps, a rocprofv3 kernel summary.
set -o pipefail
O=gpurun_out/r6b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest --maxfail=20 -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_amax.py tests/test_gpu_resblock.py tests/test_gpu_synth.py tests/test_gpu_native.py \
  tests/test_gpu_contentvec.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1
rc=$?
tail -30 $O/tests.log | grep -v "^\.\.\.\." | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stop"; exit 1; fi
grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/tests.log && { echo "GPU fault: stop"; exit 1; }
TAG=r6b/ab VARIANTS="new:RVC_X=1 noise0:RVC_AMD_FUSED_NOISE=0 fe0:RVC_AMD_FE_AMAX=0 attn0:RVC_AMD_ATTN_F16=0 ylds0:RVC_RB_YLDS=0 all0:RVC_AMD_FUSED_NOISE=0,RVC_AMD_FE_AMAX=0,RVC_AMD_ATTN_F16=0,RVC_RB_YLDS=0" R=2 bash scripts/gpu_ab_env.sh || exit 1
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/rb_stamps.py --out $O/rb_stamps.json > $O/rb_stamps.log 2>&1 || { tail -20 $O/rb_stamps.log; exit 1; }
grep -v -i warn $O/rb_stamps.log | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-per-call > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1):8 > $O/kstats.txt 2>&1 || true
head -40 $O/kstats.txt
