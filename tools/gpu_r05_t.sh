#!/bin/bash
# Analysis: the server's strict point with its colour ring in cached memory (HG_SV_DIAG_CACHED_RING, wrong images)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05t
mkdir -p $O
export HALOGEN_SERVER_GATE_TIMEOUT_MS=5000
V=$PWD/halogen-pathtracer_amd/variants
run() {  # name, lib ("" = default), args...
  local n=$1 lib=$2; shift 2
  HALOGEN_LIB=$lib timeout -k 10 120 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  echo "$n $(cut -c1-90 $O/$n.json | sed 's/.*"value": //')"
}
for i in 1 2 3; do
  run strict_base_$i "" --per-frame-only --steps 4 --server 2
  run strict_cring_$i $V/cring/libhalogen_hip.so --per-frame-only --steps 4 --server 2
done
