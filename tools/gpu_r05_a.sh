#!/bin/bash
# Round 5, first GPU pass of the render server: its tests, then the per-frame points (strict, display one behind).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_server.py -x -v --timeout 300 --timeout-method thread > $O/server_tests.log 2>&1 || { echo "server tests failed"; tail -40 $O/server_tests.log; exit 1; }
tail -3 $O/server_tests.log
for srv in 1 0; do
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server $srv > $O/strict_s$srv.json 2> $O/strict_s$srv.err || exit 1
  cat $O/strict_s$srv.json
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server $srv --display pipelined --display-format r11g11b10f --readback-depth 2 > $O/disp_s$srv.json 2> $O/disp_s$srv.err || exit 1
  cat $O/disp_s$srv.json
done
