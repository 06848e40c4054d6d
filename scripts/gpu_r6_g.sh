#!/bin/bash
# round 6, seventh GPU pass: the split-K reduces with their loads batched (f32: 8 rows per block; f64: 8 splits in
# flight); the touched suites, the default bench line (roofline, CPU baseline, per-call), the hot x6 tile's stamps and a
# kernel summary.
set -o pipefail
O=gpurun_out/r6g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest --maxfail=20 -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py tests/test_gpu_amax.py tests/test_gpu_rmvpe.py tests/test_gpu_native.py tests/test_gpu_pipeline.py \
  tests/test_gpu_configs.py tests/test_gpu_norm.py > $O/tests.log 2>&1
rc=$?
tail -30 $O/tests.log | grep -v "^\.\.\.\." | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stop"; exit 1; fi
grep -q -i -E "memory access fault|hipErrorLaunchFailure|illegal" $O/tests.log && { echo "GPU fault: stop"; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json; cut -c1-600 $O/bench.json
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --amax --only 0,6,7,8,9 \
  > $O/conv_stamps.log 2>&1 || { tail -5 $O/conv_stamps.log; exit 1; }
grep -v -E "amdgpu.ids|Warning|_warn_once" $O/conv_stamps.log | head -30
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-per-call > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1):8 > $O/kstats.txt 2>&1 || true
head -24 $O/kstats.txt
