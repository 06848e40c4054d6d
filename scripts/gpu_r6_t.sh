#!/bin/bash
# round 6: scripts/stream_stage_diff.py with the ups stages' inputs stashed and the first differing stage's difference
# mapped (channels, positions, the source term missing / doubled), fused noise on, two processes.
set -o pipefail
O=gpurun_out/r6t; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  RVC_AMD_FUSED_NOISE=1 timeout -k 10 300 python -u scripts/stream_stage_diff.py > $O/fused$r.log 2>&1 || { tail -20 $O/fused$r.log; exit 1; }
  echo "== run $r"; grep -v amdgpu.ids $O/fused$r.log | cut -c1-400
done
