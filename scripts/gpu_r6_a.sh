#!/bin/bash
# round 6, first GPU pass: the whole -m gpu suite (with the |max| producer tests, the fused source conv and the split-fp16
# attention), then an interleaved A/B of the round-6 defaults (fused noise conv + feature-extractor cells + split-fp16
# attention) against the round-5 forms, a rocprofv3 kernel summary of the default bench, and the fused ResBlock pair's
# per-tile stamps.  Results under gpurun_out/r6a.
set -o pipefail
O=gpurun_out/r6a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 780 python -u -m pytest --maxfail=30 -q --timeout 300 --timeout-method thread -m gpu tests \
  > $O/tests.log 2>&1
rc=$?
tail -40 $O/tests.log | grep -v "^\.\.\.\." | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stop"; exit 1; fi
grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/tests.log && { echo "GPU fault: stop"; exit 1; }
TAG=r6a/ab VARIANTS="new:RVC_X=1 old:RVC_AMD_FUSED_NOISE=0,RVC_AMD_FE_AMAX=0,RVC_AMD_ATTN_F16=0" R=2 bash scripts/gpu_ab_env.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-per-call > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1):8 > $O/kstats.txt 2>&1 || true
head -45 $O/kstats.txt
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/rb_stamps.py --out $O/rb_stamps.json > $O/rb_stamps.log 2>&1 || { tail -20 $O/rb_stamps.log; exit 1; }
grep -v -i warn $O/rb_stamps.log | grep -v amdgpu.ids
