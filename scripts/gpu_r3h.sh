#!/bin/bash
# full GPU suite (one process) + smoke
set -u
O=gpurun_out/${TAG:-r3h}; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -q -m gpu --maxfail=3 -rf --timeout 900 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log; cp gpurun_out/config_parity.json $O/ 2>/dev/null
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -2 $O/smoke.log; exit $rc
