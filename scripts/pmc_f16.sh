#!/bin/bash
# PMC passes (--pmc only, one run each) for the split-fp16 128x256 conv at C=128 K=11 (conv_bench shape 4)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_f16
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F16" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_f16/p$i -o run -- python3 scripts/conv_bench.py --precision f16x3 --only 4 --reps 3 > gpurun_out/pmc_f16/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i rc=$rc"; tail -5 gpurun_out/pmc_f16/p$i.log; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/pmc_f16 conv_x6
