#!/bin/bash
# Round 5: the per-frame points with the render server on and off (strict; R11G11B10F display at once and one behind)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05c
mkdir -p $O
for srv in 1 0; do
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server $srv > $O/strict_s$srv.json 2> $O/strict_s$srv.err || exit 1
  cat $O/strict_s$srv.json
  for depth in 1 2; do
    timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server $srv --display pipelined \
        --display-format r11g11b10f --readback-depth $depth > $O/disp${depth}_s$srv.json 2> $O/disp${depth}_s$srv.err || exit 1
    cat $O/disp${depth}_s$srv.json
  done
done
