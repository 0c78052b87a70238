#!/bin/bash
# Render server: XCD bands (HALOGEN_SERVER_BANDS) against the cost order, strict per-frame (forced), interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05m
mkdir -p $O
for r in 1 2; do
  for v in cost bands; do
    if [ $v = bands ]; then export HALOGEN_SERVER_BANDS=1; else unset HALOGEN_SERVER_BANDS; fi
    timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server 2 > $O/$v$r.json 2> $O/$v$r.err || { tail -3 $O/$v$r.err; exit 1; }
    echo "$v $r $(cut -c1-110 $O/$v$r.json)"
  done
done
