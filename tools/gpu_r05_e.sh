#!/bin/bash
# Kernel trace of the render server at the per-frame point: strict, and the R11G11B10F display at once (depth 1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05e
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/strict -o pf --output-format csv -- \
    python3 bench.py --per-frame-only --steps 2 --server 1 > $O/strict.log 2>&1 || { tail -5 $O/strict.log; exit 1; }
grep per_frame_only $O/strict.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/disp1 -o pf --output-format csv -- \
    python3 bench.py --per-frame-only --steps 2 --server 1 --display pipelined --display-format r11g11b10f \
    --readback-depth 1 > $O/disp1.log 2>&1 || { tail -5 $O/disp1.log; exit 1; }
grep per_frame_only $O/disp1.log
