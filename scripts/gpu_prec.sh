set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_crepe.py tests/test_gpu_ops.py > gpurun_out/pytest_prec.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_prec.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/prec_check.py pipeline_48k_v2 > gpurun_out/prec.log 2>&1 || exit $?
cat gpurun_out/prec.log
for pr in fp32 bf16x3 bf16; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --precision $pr > gpurun_out/bench_$pr.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$pr.log | cut -c1-400
done
