#!/bin/bash
# round 6: the stream use-after-free with the noise source pass -- does releasing the allocator's cached blocks after
# the per-call references, or running the per-call f0 on the fside stream (RVC_AMD_SIDE_PRIORITY=0), avoid it?
set -o pipefail
O=gpurun_out/r6r; mkdir -p $O
export TMPDIR=/tmp
RVC_AMD_FUSED_NOISE=1 timeout -k 10 300 python -u scripts/stream_diff.py --reps 2 --empty-cache > $O/ec.log 2>&1 || { tail -20 $O/ec.log; exit 1; }
echo "== empty_cache"; grep -E "^rep" $O/ec.log | cut -c1-130
RVC_AMD_FUSED_NOISE=1 RVC_AMD_SIDE_PRIORITY=0 timeout -k 10 300 python -u scripts/stream_diff.py --reps 2 > $O/sp0.log 2>&1 || { tail -20 $O/sp0.log; exit 1; }
echo "== side priority 0"; grep -E "^rep" $O/sp0.log | cut -c1-130
