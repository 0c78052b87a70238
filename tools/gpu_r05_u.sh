#!/bin/bash
# Analysis: the server's colour ring in fine-grained device memory (HALOGEN_SERVER_RING_FINEGRAINED=1): server tests, strict
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05u
mkdir -p $O
export HALOGEN_SERVER_GATE_TIMEOUT_MS=5000
HALOGEN_SERVER_RING_FINEGRAINED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py -x -v --timeout 120 --timeout-method thread > $O/server_fg.log 2>&1; echo "server tests (fine-grained ring) rc=$? $(tail -1 $O/server_fg.log)"
run() {  # name, fine-grained (0/1), args...
  local n=$1 fg=$2; shift 2
  HALOGEN_SERVER_RING_FINEGRAINED=$fg timeout -k 10 120 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  echo "$n $(cut -c1-90 $O/$n.json | sed 's/.*"value": //')"
}
for i in 1 2 3; do
  run strict_uc_$i 0 --per-frame-only --steps 4 --server 2
  run strict_fg_$i 1 --per-frame-only --steps 4 --server 2
done
