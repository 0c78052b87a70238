#!/bin/bash
# Tile-major render server: its tests, then strict / display points (server forced on, automatic, off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05j
mkdir -p $O
export HALOGEN_SERVER_GATE_TIMEOUT_MS=5000
timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py -x -v --timeout 120 --timeout-method thread > $O/server.log 2>&1 || { echo "server tests failed"; grep -E "PASS|FAIL|Error|assert" $O/server.log | tail -30; exit 1; }
tail -1 $O/server.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  echo "$n $(cut -c1-230 $O/$n.json)"
}
run strict_s2 --server 2
run strict_s1 --server 1
run disp1_s2 --server 2 --display pipelined --display-format r11g11b10f --readback-depth 1
run disp2_s2 --server 2 --display pipelined --display-format r11g11b10f --readback-depth 2
run disp2_s1 --server 1 --display pipelined --display-format r11g11b10f --readback-depth 2
