#!/bin/bash
# round 6: where the clip stream departs from the per-call form (scripts/stream_diff.py), fused noise on and off.
set -o pipefail
O=gpurun_out/r6n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/stream_diff.py > $O/sd_fused.log 2>&1 || { tail -20 $O/sd_fused.log; exit 1; }
grep -v amdgpu.ids $O/sd_fused.log
RVC_AMD_FUSED_NOISE=0 timeout -k 10 300 python -u scripts/stream_diff.py > $O/sd_unfused.log 2>&1 || { tail -20 $O/sd_unfused.log; exit 1; }
grep -v amdgpu.ids $O/sd_unfused.log
