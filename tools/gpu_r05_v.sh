#!/bin/bash
# Write-through (sc1) colour stores into a cached ring: the server tests, then strict against the uncached-ring library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05v
mkdir -p $O
export HALOGEN_SERVER_GATE_TIMEOUT_MS=5000
timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py -x -v --timeout 120 --timeout-method thread > $O/server.log 2>&1 || { echo "server tests failed"; grep -E "FAIL|Error|differ" $O/server.log | tail -10; exit 1; }
tail -1 $O/server.log
UC=$PWD/halogen-pathtracer_amd/variants/uc/libhalogen_hip.so
run() {  # name, lib ("" = default), args...
  local n=$1 lib=$2; shift 2
  HALOGEN_LIB=$lib timeout -k 10 120 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  echo "$n $(cut -c1-90 $O/$n.json | sed 's/.*"value": //')"
}
for i in 1 2 3; do
  run strict_wt_$i "" --per-frame-only --steps 4 --server 2
  run strict_uc_$i $UC --per-frame-only --steps 4 --server 2
done
run disp8_wt "" --per-frame-only --steps 4 --server 1 --display pipelined --display-format r11g11b10f --readback-depth 8
run disp8_uc $UC --per-frame-only --steps 4 --server 1 --display pipelined --display-format r11g11b10f --readback-depth 8
