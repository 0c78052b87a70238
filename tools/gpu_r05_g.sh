#!/bin/bash
# Render server after scalar polling: waves per SIMD 5 / 4, strict and R11G11B10F display at once / one behind, and the
# server off beside them
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05g
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 "$@" > $O/$n.json 2> $O/$n.err || exit 1
  echo "$n $(cut -c1-210 $O/$n.json)"
}
for w in 5 4; do
  export HALOGEN_SERVER_WAVES=$w
  run strict_w$w --server 1
  run disp1_w$w --server 1 --display pipelined --display-format r11g11b10f --readback-depth 1
  run disp2_w$w --server 1 --display pipelined --display-format r11g11b10f --readback-depth 2
done
unset HALOGEN_SERVER_WAVES
run strict_off --server 0
run disp1_off --server 0 --display pipelined --display-format r11g11b10f --readback-depth 1
run disp2_off --server 0 --display pipelined --display-format r11g11b10f --readback-depth 2
