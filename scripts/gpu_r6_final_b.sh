#!/bin/bash
# round 6, end of round (2/2): rocprofv3 kernel stats of the default bench command, PMC traffic on this tree (separate
# FETCH_SIZE / WRITE_SIZE passes), the hot conv's and the fused pairs' stamps, the cfg 3 / cfg 5 bench lines.
set -o pipefail
O=gpurun_out/r6final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  > $O/bench_rocprof.log 2>&1 || { tail -20 $O/bench_rocprof.log; exit 1; }
grep '^{' $O/bench_rocprof.log | tail -1 | cut -c1-200
python scripts/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1):15 > $O/kstats.txt 2>&1 || true
head -12 $O/kstats.txt
bash scripts/pmc_traffic.sh > $O/pmc_traffic.log 2>&1 || { tail -20 $O/pmc_traffic.log; exit 1; }
tail -6 $O/pmc_traffic.log
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --amax --only 0,6,7,8,9 \
  --out $O/conv_stamps.json > $O/conv_stamps.log 2>&1 || { tail -5 $O/conv_stamps.log; exit 1; }
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 200 python -u scripts/rb_stamps.py --out $O/rb_stamps.json \
  > $O/rb_stamps.log 2>&1 || { tail -5 $O/rb_stamps.log; exit 1; }
grep -E "^c(32|64)" $O/rb_stamps.log | cut -c1-120
timeout -k 10 400 python -u bench.py --chunks 64 --seconds 10 --index-rate 0.75 --precision bf16x3 --batch 8 --steps 5 \
  --warmup 2 --no-cpu-baseline > $O/bench_cfg3.log 2>&1 || { tail -20 $O/bench_cfg3.log; exit 1; }
grep '^{' $O/bench_cfg3.log | tail -1 | cut -c1-160
timeout -k 10 400 python -u bench.py --sr 40000 --f0 crepe-full --precision bf16x3 --graph --chunks 4 --steps 5 --warmup 2 \
  --no-cpu-baseline > $O/bench_cfg5.log 2>&1 || { tail -20 $O/bench_cfg5.log; exit 1; }
grep '^{' $O/bench_cfg5.log | tail -1 | cut -c1-160
