#!/bin/bash
set -u
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u scripts/rmvpe_prec.py 30 201 > gpurun_out/r3c/prec.log 2>&1 || { tail -20 gpurun_out/r3c/prec.log; exit 1; }
tail -14 gpurun_out/r3c/prec.log
RVC_AMD_X6=0 timeout -k 10 300 python -u scripts/rmvpe_prec.py 30 201 > gpurun_out/r3c/prec_f32engine.log 2>&1 || { tail -20 gpurun_out/r3c/prec_f32engine.log; exit 1; }
tail -14 gpurun_out/r3c/prec_f32engine.log
