#!/bin/bash
# PMC on the f64 conv engine's MFMA-only loop (C64_DBG 15) and the whole kernel, 16x16x4 (m0) vs 4x4x4 (m1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4l; mkdir -p $O
export LD_LIBRARY_PATH=$PWD/rvc-maker_amd/lib:$LD_LIBRARY_PATH
for v in 0_m0 0_m1 15_m0 15_m1; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/$v/p1 -o run -- scripts/conv64_dbg_$v 128 376 16 9 4 1 > $O/p$v.log 2>&1 || { echo "pmc $v failed"; tail -3 $O/p$v.log; exit 1; }
  grep dbg $O/p$v.log
  python3 scripts/pmc_summary.py $O/$v conv64_kernel
done
