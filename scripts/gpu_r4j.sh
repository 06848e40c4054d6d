#!/bin/bash
# kernel trace + stats of the bench's clip stream (3 timed steps), grouped by kernel and grid.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bs -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-per-call > $O/bs.log 2>&1 || { echo "rocprof failed"; tail -5 $O/bs.log; exit 1; }
grep '"metric"' $O/bs.log | cut -c1-200
python3 scripts/kstats.py $O/bs/run_kernel_stats.csv:4 > $O/kstats.txt; head -40 $O/kstats.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_configs.py > $O/t_cfg.log 2>&1 || { tail -30 $O/t_cfg.log; exit 1; }
tail -2 $O/t_cfg.log; ls gpurun_out/*.json
