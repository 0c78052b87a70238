#!/bin/bash
# Per-frame device timing of the render server (analysis build HG_SV_DIAG_TIMES): display one frame behind and strict
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05q
mkdir -p $O
export HALOGEN_LIB=$PWD/halogen-pathtracer_amd/variants/diag/libhalogen_hip.so HALOGEN_SERVER_TRACE=1
timeout -k 10 120 python -u bench.py --per-frame-only --steps 1 --server 2 --display pipelined --display-format r11g11b10f \
    --readback-depth 2 > $O/d2.json 2> $O/d2.err || { tail -3 $O/d2.err; exit 1; }
grep -c "first claim" $O/d2.err
timeout -k 10 120 python -u bench.py --per-frame-only --steps 1 --server 2 > $O/s.json 2> $O/s.err || { tail -3 $O/s.err; exit 1; }
grep -c "first claim" $O/s.err
