#!/bin/bash
# clip-stream variants on one box: groups of B clips (batched front end + synthesizer), stream priorities
set -u
O=gpurun_out/${TAG:-svar}; mkdir -p $O
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --no-per-call --steps 20 --warmup 4 $BARGS > $O/$name.log 2>&1 || { tail -3 $O/$name.log; exit 1; }
  echo "$name $(grep -o '"value": [0-9.]*' $O/$name.log | head -1)"
}
BARGS="" run b1 RVC_X=0
BARGS="--batch 2" run b2 RVC_X=0
BARGS="--batch 4" run b4 RVC_X=0
BARGS="" run b1_fside_hi RVC_AMD_FSIDE_PRIORITY=-1
BARGS="" run b1_back_norm RVC_AMD_BACK_PRIORITY=0
BARGS="--batch 2" run b2_fside_hi RVC_AMD_FSIDE_PRIORITY=-1
BARGS="" run b1_again RVC_X=0
