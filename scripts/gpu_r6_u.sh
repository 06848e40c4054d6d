#!/bin/bash
# round 6: the stream race with split-K off everywhere (RVC_SPLITK_TILES=0: no reduce launch between the transposed conv
# and the source pass), fused noise on, two processes (scripts/stream_stage_diff.py).
set -o pipefail
O=gpurun_out/r6u; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  RVC_SPLITK_TILES=0 RVC_AMD_FUSED_NOISE=1 timeout -k 10 300 python -u scripts/stream_stage_diff.py > $O/nosplit$r.log 2>&1 || { tail -20 $O/nosplit$r.log; exit 1; }
  echo "== run $r"; grep -v amdgpu.ids $O/nosplit$r.log | cut -c1-300
done
