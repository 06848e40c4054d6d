#!/bin/bash
# PMC counter passes (separate runs, --pmc only with kernel dispatch info) for one conv_bench shape set.
# usage: scripts/pmc.sh TAG "bench args"
set -u
TAG=${1:?tag}; ARGS=${2:-}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_$TAG/p$i -o run -- python3 scripts/conv_bench.py $ARGS > gpurun_out/pmc_$TAG/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i rc=$rc"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit $rc; fi
done
echo pmc done
