#!/bin/bash
# round 6, first GPU pass: the |max| producer tests, the fused source conv, the suites the round-6 kernel changes touch,
# then an interleaved A/B of the new defaults (fused noise conv + feature-extractor cells) against the round-5 forms
# and a rocprofv3 kernel summary of the default bench.  Results under gpurun_out/r6a.
set -o pipefail
O=gpurun_out/r6a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest --maxfail=20 -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_amax.py tests/test_gpu_ops.py tests/test_gpu_synth.py tests/test_gpu_contentvec.py \
  tests/test_gpu_native.py tests/test_gpu_batch.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
TAG=r6a/ab VARIANTS="new:RVC_X=1 old:RVC_AMD_FUSED_NOISE=0,RVC_AMD_FE_AMAX=0" R=2 bash scripts/gpu_ab_env.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-per-call > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1):8 > $O/kstats.txt 2>&1 || true
head -45 $O/kstats.txt
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/rb_stamps.py --out $O/rb_stamps.json > $O/rb_stamps.log 2>&1 || { tail -20 $O/rb_stamps.log; exit 1; }
grep -v -i warn $O/rb_stamps.log | grep -v amdgpu.ids
