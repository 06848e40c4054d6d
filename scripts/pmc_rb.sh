#!/bin/bash
# PMC passes (one rocprofv3 run each, --pmc only) over the fused ResBlock pair shapes (scripts/rb_bench.py)
set -u
TAG=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_$TAG/p$i -o run -- python3 scripts/rb_bench.py --reps 1 > gpurun_out/pmc_$TAG/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i rc=$rc"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit $rc; fi
done
echo pmc done
