#!/bin/bash
# round 6: the stage of the clip stream's synthesizer where the fused-noise stream departs from the per-call form
# (scripts/stream_stage_diff.py), fused noise on (r6s also ran it with the pass off: no stage differs).
set -o pipefail
O=gpurun_out/r6s; mkdir -p $O
export TMPDIR=/tmp
RVC_AMD_FUSED_NOISE=1 timeout -k 10 300 python -u scripts/stream_stage_diff.py > $O/fused.log 2>&1 || { tail -20 $O/fused.log; exit 1; }
echo "== fused"; grep -E "clip" $O/fused.log


