#!/bin/bash
# Render server A/B: its tests, then strict per-frame (forced) twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py -x -q --timeout 120 --timeout-method thread > $O/server.log 2>&1 || { echo "server tests failed"; tail -30 $O/server.log; exit 1; }
tail -1 $O/server.log
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server 2 > $O/strict$r.json 2> $O/strict$r.err || { tail -3 $O/strict$r.err; exit 1; }
  echo "strict $r $(cut -c1-120 $O/strict$r.json)"
done
