#!/bin/bash
# Rehearsal of the driver's N=2 launch on the one-GPU box (both ranks share cuda:0): the default bench line.
set -o pipefail
O=gpurun_out/r4n2; mkdir -p $O
HIP_VISIBLE_DEVICES=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/n2.log 2>&1
rc=$?; grep '"metric"' $O/n2.log | cut -c1-400; tail -3 $O/n2.log; exit $rc
