#!/bin/bash
# round 5: ContentVec's K = 1 GEMMs in split-fp16 from the producers' |max| (LayerNorm / attention / fc1 cells) --
# ContentVec, native-host, batch and config tests, bench A/B
set -o pipefail
O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_contentvec.py tests/test_gpu_embedder_st.py tests/test_gpu_batch.py tests/test_gpu_native.py tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_ops.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
cp gpurun_out/config_parity.json $O/ 2>/dev/null || true
for r in 1 2; do
for f in 0 1; do
RVC_AMD_CV_AMAX=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${f}_${r}.log 2>&1 || { tail -20 $O/b_${f}_${r}.log; exit 1; }
echo "cv_amax=$f $(tail -1 $O/b_${f}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
