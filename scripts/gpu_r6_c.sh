#!/bin/bash
# round 6, third GPU pass: the TextEncoder / flow |max| cells, the 128-byte-row x6 epilogue (permlane16 swap), the
# source pass with LDS-staged weights; the touched suites, then an interleaved per-feature A/B (each default off alone)
# and a rocprofv3 kernel summary.
set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest --maxfail=20 -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py tests/test_gpu_amax.py tests/test_gpu_resblock.py tests/test_gpu_synth.py tests/test_gpu_native.py \
  tests/test_gpu_pipeline.py tests/test_gpu_configs.py > $O/tests.log 2>&1
rc=$?
tail -30 $O/tests.log | grep -v "^\.\.\.\." | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stop"; exit 1; fi
grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/tests.log && { echo "GPU fault: stop"; exit 1; }
TAG=r6c/ab VARIANTS="new:RVC_X=1 swz0:RVC_X6_SWZ=0 te0:RVC_AMD_TE_AMAX=0 noise0:RVC_AMD_FUSED_NOISE=0 ylds0:RVC_RB_YLDS=0 attn0:RVC_AMD_ATTN_F16=0" R=2 bash scripts/gpu_ab_env.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-per-call > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1):8 > $O/kstats.txt 2>&1 || true
head -40 $O/kstats.txt
