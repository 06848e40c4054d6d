#!/bin/bash
# PMC passes (one counter set per rocprofv3 run) on the two hottest shapes: the split-fp16 C = 128 K = 11 conv
# (conv_bench shape 4) and the fused ResBlock pairs (rb_bench).  Summaries in $O/summary_*.txt.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmchot}; mkdir -p $O
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VALU_MFMA_MOPS_F16")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/pc$i -o run -- python3 scripts/conv_bench.py --only 4 --reps 3 ${CB_ARGS:-} > $O/c$i.log 2>&1 || { echo "conv pass $i failed"; tail -3 $O/c$i.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc $set --output-format csv -d $O/pr$i -o run -- python3 scripts/rb_bench.py --reps 2 > $O/r$i.log 2>&1 || { echo "rb pass $i failed"; tail -3 $O/r$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $O conv_x6 > $O/summary_conv.txt; python3 scripts/pmc_summary.py $O resblock_x6 > $O/summary_rb.txt
cat $O/summary_conv.txt $O/summary_rb.txt
