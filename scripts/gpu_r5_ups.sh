#!/bin/bash
# round 5: the upsampling convs' inputs through |max| cells (split-fp16 for ups[0..2]) -- synth / pipeline / native /
# config / batch tests, bench A/B
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_synth.py tests/test_gpu_native.py tests/test_gpu_pipeline.py tests/test_gpu_batch.py tests/test_gpu_configs.py tests/test_gpu_convert.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
cp gpurun_out/config_parity.json $O/ 2>/dev/null || true
for r in 1 2; do
for f in 0 1; do
RVC_AMD_AMAX_UPS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${f}_${r}.log 2>&1 || { tail -20 $O/b_${f}_${r}.log; exit 1; }
echo "amax_ups=$f $(tail -1 $O/b_${f}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
