#!/bin/bash
# Render server waves per SIMD: strict and R11G11B10F display (at once / one behind), server on (waves 5, 4, 3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05d
mkdir -p $O
for w in 5 4; do
  export HALOGEN_SERVER_WAVES=$w
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server 1 > $O/strict_w$w.json 2> $O/strict_w$w.err || exit 1
  echo "w=$w strict $(cat $O/strict_w$w.json)"
  for depth in 1 2; do
    timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server 1 --display pipelined \
        --display-format r11g11b10f --readback-depth $depth > $O/disp${depth}_w$w.json 2> $O/disp${depth}_w$w.err || exit 1
    echo "w=$w depth $depth $(cat $O/disp${depth}_w$w.json)"
  done
done
