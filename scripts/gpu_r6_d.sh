#!/bin/bash
# round 6, fourth GPU pass: grouped convs on the split-operand engine (ContentVec's pos_conv, one group per phase), the
# TextEncoder / flow |max| cells split into two switches; the touched suites, the synthesizer's stages alone per switch
# (scripts/synth_stage_time.py), an interleaved end-to-end A/B and a rocprofv3 kernel summary.
set -o pipefail
O=gpurun_out/r6d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest --maxfail=20 -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py tests/test_gpu_amax.py tests/test_gpu_contentvec.py tests/test_gpu_native.py \
  tests/test_gpu_pipeline.py tests/test_gpu_synth.py > $O/tests.log 2>&1
rc=$?
tail -30 $O/tests.log | grep -v "^\.\.\.\." | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stop"; exit 1; fi
grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/tests.log && { echo "GPU fault: stop"; exit 1; }
timeout -k 10 300 python -u scripts/synth_stage_time.py --out $O/synth_stages.json base TE_AMAX=0 FLOW_AMAX=0 \
  TE_AMAX=0,FLOW_AMAX=0 ATTN_F16=0 FUSED_NOISE=0 > $O/synth_stages.log 2>&1 || { tail -5 $O/synth_stages.log; exit 1; }
cat $O/synth_stages.log | grep -v amdgpu.ids
TAG=r6d/ab VARIANTS="new:RVC_X=1 te0:RVC_AMD_TE_AMAX=0 flow0:RVC_AMD_FLOW_AMAX=0 both0:RVC_AMD_TE_AMAX=0,RVC_AMD_FLOW_AMAX=0 grp0:RVC_X6_GROUPED=0" R=2 bash scripts/gpu_ab_env.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-per-call > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1):8 > $O/kstats.txt 2>&1 || true
head -32 $O/kstats.txt
