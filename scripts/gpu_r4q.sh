#!/bin/bash
# Winograd per-image rule: op tests, RMVPE f64 time per RVC_RMVPE_WINO_MINP, bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "wino or conv64 or bordered" > $O/t_ops.log 2>&1 || { tail -30 $O/t_ops.log; exit 1; }
tail -1 $O/t_ops.log
for mp in 0 90 300 1000; do
  RVC_RMVPE_WINO_MINP=$mp timeout -k 10 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rm$mp.log 2>&1 || { tail $O/rm$mp.log; exit 1; }
  echo "minp $mp $(tail -1 $O/rm$mp.log)"
done
RVC_RMVPE_WINO=0 timeout -k 10 200 python -u scripts/rmvpe_prof.py f64 5 > $O/rmoff.log 2>&1 && echo "off $(tail -1 $O/rmoff.log)"
TAG=r4q/ab R=2 VARIANTS="mp0:RVC_RMVPE_WINO_MINP=0 mp90:RVC_RMVPE_WINO_MINP=90 mp300:RVC_RMVPE_WINO_MINP=300 off:RVC_RMVPE_WINO=0" ./scripts/gpu_ab_env.sh
