#!/bin/bash
# Render server variants (ring 32; faster host polling), strict per-frame (forced), interleaved with the shipped library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05n
mkdir -p $O
for r in 1 2; do
  for v in shipped nb; do
    if [ $v = shipped ]; then unset HALOGEN_LIB; else export HALOGEN_LIB=$PWD/halogen-pathtracer_amd/variants/$v/libhalogen_hip.so; fi
    timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server 2 > $O/$v$r.json 2> $O/$v$r.err || { tail -3 $O/$v$r.err; exit 1; }
    echo "$v $r $(cut -c1-110 $O/$v$r.json)"
  done
done
