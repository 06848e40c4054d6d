#!/bin/bash
# PMC passes (one rocprofv3 run each, --pmc only) over conv_bench shapes; usage: pmc_conv.sh TAG "bench args"
set -u
TAG=${1:?tag}; ARGS=${2:-}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
i=0
for set in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_$TAG/p$i -o run -- python3 scripts/conv_bench.py $ARGS > gpurun_out/pmc_$TAG/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i rc=$rc"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit $rc; fi
done
echo pmc done
