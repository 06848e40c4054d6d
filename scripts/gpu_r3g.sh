#!/bin/bash
# A/B: in-launch split-K reduce vs separate pass; RMVPE split-accumulator vs 6-pass (same box)
set -u
O=gpurun_out/r3g; mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['per_call']['value'], r['kernel_ms_per_step'], {k:(v['launches'],v['kernel_ms']) for k,v in r['by_pass_set'].items()})"; }
run fused_sa RVC_SPLITK_FUSED=1
run sep_sa RVC_SPLITK_FUSED=0
run sep_x6 RVC_SPLITK_FUSED=0 RVC_RMVPE_PRECISION=fp32
run fused_x6 RVC_SPLITK_FUSED=1 RVC_RMVPE_PRECISION=fp32
run sep_sa2 RVC_SPLITK_FUSED=0
