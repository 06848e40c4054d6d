#!/bin/bash
# PMC passes over ContentVec's 3072 x 768 x 1599 K = 1 GEMM (split-K off), one rocprofv3 run per counter set
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmcg}; mkdir -p $O
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM" "FETCH_SIZE"; do
  i=$((i+1))
  RVC_SPLITK_TILES=0 timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 scripts/gemm_bench.py --child fp32 --only 0 --reps 3 > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i rc=$rc"; tail -5 $O/p$i.log; exit $rc; fi
done
python3 scripts/pmc_summary.py $O conv_x6
