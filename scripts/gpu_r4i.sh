#!/bin/bash
# planner check, RMVPE f64 time, 1-GPU bench, the cfg 4 2-rank shared-GPU rehearsal, the cpu_baseline thread scan.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 120 python -u scripts/conv64_sweep.py $O/planner.json --planner-only > $O/planner.log 2>&1 || { tail $O/planner.log; exit 1; }
grep planner $O/planner.log
timeout -k 10 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rm.log 2>&1 || { tail $O/rm.log; exit 1; }
tail -1 $O/rm.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --utterances 120 --seconds 30 --no-cpu-baseline --no-roofline > $O/cfg4_2rank.log 2>&1 || { tail $O/cfg4_2rank.log; exit 1; }
grep '"metric"' $O/cfg4_2rank.log | cut -c1-400
timeout -k 10 600 python -u scripts/cpu_threads.py 8 16 32 64 > $O/cpu_threads.log 2>&1 || { tail $O/cpu_threads.log; exit 1; }
tail -3 $O/cpu_threads.log
TAG=r4i/pmchot ./scripts/gpu_pmc_hot.sh > $O/pmchot.log 2>&1 || { tail $O/pmchot.log; exit 1; }
tail -2 $O/pmchot.log | cut -c1-600
