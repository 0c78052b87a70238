#!/bin/bash
# Idle-sleep variants of the render server: display at once (depth 1) and strict, kernel trace of display
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05f
mkdir -p $O
for v in shipped s8 s32; do
  if [ $v = shipped ]; then unset HALOGEN_LIB; else export HALOGEN_LIB=$PWD/halogen-pathtracer_amd/variants/$v/libhalogen_hip.so; fi
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 2 --server 1 --display pipelined --display-format r11g11b10f \
      --readback-depth 1 > $O/disp1_$v.json 2> $O/disp1_$v.err || exit 1
  echo "$v depth1 $(cut -c1-200 $O/disp1_$v.json)"
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 2 --server 1 > $O/strict_$v.json 2> $O/strict_$v.err || exit 1
  echo "$v strict $(cut -c1-200 $O/strict_$v.json)"
done
