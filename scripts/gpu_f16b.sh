#!/bin/bash
# split-fp16 vs split-bf16 x6: fused resblock pairs and the pipeline branches under each precision
set -u
mkdir -p gpurun_out
for prec in fp32 f16x3; do
  timeout -k 10 200 python scripts/rb_bench.py --precision $prec > gpurun_out/rb_$prec.log 2>&1 || { tail gpurun_out/rb_$prec.log; exit 1; }
  echo "== rb $prec"; tail -8 gpurun_out/rb_$prec.log
  RVC_AMD_PRECISION=$prec timeout -k 10 200 python scripts/micro.py branches > gpurun_out/br_$prec.log 2>&1 || { tail gpurun_out/br_$prec.log; exit 1; }
  echo "== branches $prec"; tail -6 gpurun_out/br_$prec.log
done
