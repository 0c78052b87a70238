#!/bin/bash
# Server strict point against the streaming kernel's deep-scene thresholds (variant builds; batched C3 beside it)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05s
mkdir -p $O
export HALOGEN_SERVER_GATE_TIMEOUT_MS=5000
V=$PWD/halogen-pathtracer_amd/variants
run() {  # name, lib ("" = default), args...
  local n=$1 lib=$2; shift 2
  HALOGEN_LIB=$lib timeout -k 10 120 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  echo "$n $(cut -c1-90 $O/$n.json | sed 's/.*"value": //')"
}
for i in 1 2; do
  for v in base t16 t24 t28 r20 r32; do
    lib=""; [ $v = base ] || lib=$V/$v/libhalogen_hip.so
    run strict_${v}_$i "$lib" --per-frame-only --steps 4 --server 2
  done
done
for v in base t24 r32; do
  lib=""; [ $v = base ] || lib=$V/$v/libhalogen_hip.so
  run batched_$v "$lib" --steps 8 --warmup 2 --no-cpu-baseline --no-framed --no-per-frame --no-counters
done
