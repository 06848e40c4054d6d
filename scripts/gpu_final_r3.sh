#!/bin/bash
# Round-3 final: the whole -m gpu suite and smoke, the artifact set (bench line, rocprof stats, PMC traffic,
# stream timeline), and the BASELINE cfg 3 / cfg 5 bench variants.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fin3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
TAG=${TAG:-fin3}_art bash scripts/gpu_art_r3.sh || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-roofline --chunks 64 --seconds 10 --index-rate 0.75 --precision bf16x3 --batch 8 --steps 2 --warmup 1 > $O/cfg3.log 2>&1 || { tail -3 $O/cfg3.log; exit 1; }
echo "cfg3 $(grep -o '"value": [0-9.]*' $O/cfg3.log | head -2 | tr '\n' ' ')"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-roofline --sr 40000 --f0 crepe-full --precision bf16x3 --graph --chunks 4 --steps 3 --warmup 1 > $O/cfg5.log 2>&1 || { tail -3 $O/cfg5.log; exit 1; }
echo "cfg5 $(grep -o '"value": [0-9.]*' $O/cfg5.log | head -1)"
