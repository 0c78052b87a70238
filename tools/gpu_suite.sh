#!/bin/bash
# The whole -m gpu suite (server tests first) and the smoke, one process per step, progress per test in
# gpurun_out/suite/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/suite
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_server.py -x -v --timeout 240 --timeout-method thread > $O/server.log 2>&1 || { echo "server tests failed"; tail -30 $O/server.log; exit 1; }
tail -1 $O/server.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread --deselect tests/test_gpu_server.py > $O/all.log 2>&1; rc=$?
tail -2 $O/all.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/all.log | head -20; exit $rc; }
