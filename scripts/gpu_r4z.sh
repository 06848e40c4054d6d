#!/bin/bash
# A/B: B-operand LDS reads pinned one fragment ahead (X6_BPIN / RB_BPIN) vs the default build.
set -o pipefail
O=gpurun_out/r4z; mkdir -p $O
V=rvc-maker_amd/lib/bpin/librvc_amd.so
timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 > $O/conv_base.log 2>&1 && \
RVC_AMD_LIB=$V timeout -k 10 300 python -u scripts/conv_bench.py --reps 10 > $O/conv_bpin.log 2>&1 && \
timeout -k 10 300 python -u scripts/rb_bench.py > $O/rb_base.log 2>&1 && \
RVC_AMD_LIB=$V timeout -k 10 300 python -u scripts/rb_bench.py > $O/rb_bpin.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_base.log 2>&1 && \
RVC_AMD_LIB=$V timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_bpin.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_base2.log 2>&1 && \
RVC_AMD_LIB=$V timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_bpin2.log 2>&1
rc=$?
for f in conv_base conv_bpin rb_base rb_bpin; do echo == $f; tail -12 $O/$f.log; done
for f in bench_base bench_bpin bench_base2 bench_bpin2; do grep '"metric"' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['per_call'])"; done
exit $rc
