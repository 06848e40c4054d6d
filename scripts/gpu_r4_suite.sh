#!/bin/bash
# The driver's round-end GPU tiers on the final tree: the -m gpu suite, then smoke().
set -o pipefail
O=gpurun_out/suite_final; mkdir -p $O
timeout -k 10 2400 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/gpu_suite.log 2>&1 || { tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 600 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
