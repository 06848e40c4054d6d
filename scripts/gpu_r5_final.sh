#!/bin/bash
# round 5, end of round: smoke, default bench lines, rocprofv3 kernel stats of the bench, PMC traffic, hot-kernel PMC,
# conv precision on the generator's shapes, conv stamps.  Results under gpurun_out/r5final (copied into profiles/).
set -o pipefail
O=gpurun_out/r5final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
timeout -k 10 400 python -u bench.py > $O/bench_$r.log 2>&1 || { tail -20 $O/bench_$r.log; exit 1; }
tail -1 $O/bench_$r.log | cut -c1-400
done
bash scripts/gpu_prof.sh r5 || exit 1
bash scripts/pmc_traffic.sh > $O/pmc_traffic.log 2>&1 || { tail -20 $O/pmc_traffic.log; exit 1; }
tail -5 $O/pmc_traffic.log
TAG=r5pmchot bash scripts/gpu_pmc_hot.sh > $O/pmchot.log 2>&1 || { tail -20 $O/pmchot.log; exit 1; }
tail -12 $O/pmchot.log
timeout -k 10 300 python -u scripts/conv_prec.py --gen --out $O/conv_prec_gen.txt > $O/conv_prec.log 2>&1 || { tail -20 $O/conv_prec.log; exit 1; }
cat $O/conv_prec_gen.txt
RVC_AMD_LIB=rvc-maker_amd/lib/s/librvc_amd.so timeout -k 10 300 python -u scripts/conv_stamps.py --amax --only 0,1,2,3,7,8,9,10 --out $O/conv_stamps.json > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -v -i warn $O/stamps.log | grep -v amdgpu.ids | head -40
