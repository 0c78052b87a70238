#!/bin/bash
# Several units per claim (HG_SV_CLAIM; default 2): the server tests (default and 8), then strict / display points
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05r2
mkdir -p $O
export HALOGEN_SERVER_GATE_TIMEOUT_MS=5000
V=$PWD/halogen-pathtracer_amd/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py -x -v --timeout 120 --timeout-method thread > $O/server.log 2>&1 || { echo "server tests failed"; grep -E "PASS|FAIL|Error|assert" $O/server.log | tail -30; exit 1; }
tail -1 $O/server.log
HALOGEN_LIB=$V/claim8/libhalogen_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py -x -v --timeout 120 --timeout-method thread > $O/server8.log 2>&1 || { echo "server tests (claim 8) failed"; grep -E "PASS|FAIL|Error|assert" $O/server8.log | tail -30; exit 1; }
tail -1 $O/server8.log
run() {  # name, lib ("" = default), args...
  local n=$1 lib=$2; shift 2
  HALOGEN_LIB=$lib timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  echo "$n $(cut -c1-90 $O/$n.json)"
}
for i in 1 2; do
  run strict2_$i "" --server 2
  run strict1_$i $V/claim1/libhalogen_hip.so --server 2
  run strict4_$i $V/claim4/libhalogen_hip.so --server 2
  run strict8_$i $V/claim8/libhalogen_hip.so --server 2
done
for c in 2 1 4 8; do
  lib=""; [ $c = 2 ] || lib=$V/claim$c/libhalogen_hip.so
  run disp1_c$c "$lib" --server 2 --display pipelined --display-format r11g11b10f --readback-depth 1
  run disp2_c$c "$lib" --server 2 --display pipelined --display-format r11g11b10f --readback-depth 2
done
