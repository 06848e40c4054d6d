#!/bin/bash
# round 6: which form is off -- the clip stream or the per-call pipeline -- against the unfused-noise synthesizer.
set -o pipefail
O=gpurun_out/r6p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/stream_diff.py --reps 2 > $O/sd.log 2>&1 || { tail -20 $O/sd.log; exit 1; }
grep -v amdgpu.ids $O/sd.log
PYTORCH_NO_CUDA_MEMORY_CACHING=1 timeout -k 10 400 python -u scripts/stream_diff.py --reps 1 > $O/sd_nocache.log 2>&1 || { tail -20 $O/sd_nocache.log; exit 1; }
grep -v amdgpu.ids $O/sd_nocache.log
