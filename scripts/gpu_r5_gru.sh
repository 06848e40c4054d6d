#!/bin/bash
# round 5: the BiGRU recurrence -- f64 vs the f32 recurrence (workgroups per direction, XCD spread): per-step time,
# output difference, the headline clip's f0 decisions, bench A/B
set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
run() { timeout -k 10 120 env "$@" > $O/last.log 2>&1 || { tail -20 $O/last.log; exit 1; }; grep -v -i warn $O/last.log | grep -v amdgpu.ids; }
run RVC_BIGRU64_F32=0 python -u scripts/bigru64_time.py --save $O/y64.npy
run RVC_BIGRU64_F32=0 RVC_BIGRU64_WG=8 python -u scripts/bigru64_time.py
run RVC_BIGRU64_F32=1 RVC_BIGRU64_MXWG=4 RVC_BIGRU64_SPREAD=1 python -u scripts/bigru64_time.py --save $O/y32.npy
run RVC_BIGRU64_F32=1 RVC_BIGRU64_MXWG=4 RVC_BIGRU64_SPREAD=0 python -u scripts/bigru64_time.py
run RVC_BIGRU64_F32=1 RVC_BIGRU64_MXWG=8 python -u scripts/bigru64_time.py
run RVC_BIGRU64_F32=1 RVC_BIGRU64_MXWG=16 python -u scripts/bigru64_time.py
python3 -c "
import numpy as np; a=np.load('$O/y64.npy'); b=np.load('$O/y32.npy'); print('f32 recurrence vs f64: max abs diff %.3e rms %.3e' % (np.abs(a-b).max(), np.sqrt(((a-b)**2).mean())))"
RVC_BIGRU64_F32=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py -k "headline" > $O/t_head.log 2>&1 || { tail -30 $O/t_head.log; exit 1; }
tail -2 $O/t_head.log
for r in 1 2; do
for f in 0 1; do
RVC_BIGRU64_F32=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --steps 12 --warmup 3 > $O/b_${f}_${r}.log 2>&1 || { tail -20 $O/b_${f}_${r}.log; exit 1; }
echo "gru_f32=$f $(tail -1 $O/b_${f}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_call"]["value"])')"
done; done
