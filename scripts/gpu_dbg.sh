set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py -k "f0_post or change_rms or opts" > gpurun_out/pytest_dbg.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_dbg.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for pr in fp32 bf16; do for d in 0 1 2 4 7; do
  echo "== precision $pr debug $d"
  RVC_CONV_DEBUG=$d timeout -k 10 120 python -u scripts/conv_bench.py --reps 5 --precision $pr > gpurun_out/cb_${pr}_$d.log 2>&1 || exit $?
  grep -E "C= 128|C=  64|total" gpurun_out/cb_${pr}_$d.log
done; done
