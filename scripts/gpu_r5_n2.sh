#!/bin/bash
# round 5: N=2 launch rehearsal of the default bench on one shared GPU (gloo gather), and the cfg 4 utterance mode
set -o pipefail
O=gpurun_out/r5n2; mkdir -p $O
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --warmup 2 --no-cpu-baseline > $O/n2.log 2>&1 || { tail -20 $O/n2.log; exit 1; }
grep '"metric"' $O/n2.log | cut -c1-400
