#!/bin/bash
# A/B: conv engine compute waves at s_setprio 2 (X6_PRIO=2, a variant build) vs default.
set -o pipefail
O=gpurun_out/r4pr; mkdir -p $O
V=rvc-maker_amd/lib/pr/librvc_amd.so
timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 > $O/conv_base.log 2>&1 && \
RVC_AMD_LIB=$V timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 --check > $O/conv_jp.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/b0.log 2>&1 && \
RVC_AMD_LIB=$V timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/b1.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/b0b.log 2>&1 && \
RVC_AMD_LIB=$V timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/b1b.log 2>&1
rc=$?; for f in conv_base conv_jp; do echo == $f; grep "C=\|total" $O/$f.log; done
for f in b0 b1 b0b b1b; do grep '"metric"' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['per_call'])"; done
exit $rc
