#!/bin/bash
# f64 MFMA rate variants, BiGRU64 variants, RMVPE f64 time with the new recurrence, one PMC pass on the f64 convs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b; mkdir -p $O
step() { local t=$1; shift; echo "== $*"; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
step 200 ./scripts/bigru64_bench 3232 > $O/bigru64_bench.log 2>&1; cat $O/bigru64_bench.log
step 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rmvpe_f64.log 2>&1; tail -1 $O/rmvpe_f64.log
step 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py -k bigru > $O/t_bigru.log 2>&1; tail -2 $O/t_bigru.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pc1 -o run -- python3 scripts/rmvpe_prof.py f64 2 > $O/pc1.log 2>&1 || { echo "pmc failed"; tail -3 $O/pc1.log; exit 1; }
python3 scripts/pmc_summary.py $O conv64_kernel > $O/summary_conv64.txt; cat $O/summary_conv64.txt
