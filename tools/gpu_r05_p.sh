#!/bin/bash
# Render server wake-up: short idle sleeps + host word polled every spin (variant "fast") against the shipped library,
# display one frame behind (forced server) and strict
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05p2
mkdir -p $O
for v in shipped; do
  if [ $v = shipped ]; then unset HALOGEN_LIB; else export HALOGEN_LIB=$PWD/halogen-pathtracer_amd/variants/$v/libhalogen_hip.so; fi
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server 2 --display pipelined --display-format r11g11b10f --readback-depth 2 > $O/d2_$v.json 2> $O/d2_$v.err || { tail -3 $O/d2_$v.err; exit 1; }
  echo "$v one-behind $(cut -c1-110 $O/d2_$v.json)"
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server 2 --display pipelined --display-format r11g11b10f --readback-depth 1 > $O/d1_$v.json 2> $O/d1_$v.err || { tail -3 $O/d1_$v.err; exit 1; }
  echo "$v at-once $(cut -c1-110 $O/d1_$v.json)"
  timeout -k 10 120 python -u bench.py --per-frame-only --steps 4 --server 2 > $O/s_$v.json 2> $O/s_$v.err || { tail -3 $O/s_$v.err; exit 1; }
  echo "$v strict $(cut -c1-110 $O/s_$v.json)"
done
