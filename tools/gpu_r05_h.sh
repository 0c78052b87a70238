#!/bin/bash
# Timelines (kernels + copies) of the R11G11B10F display one frame behind, render server on and off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05h
mkdir -p $O
for srv in 1 0; do
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $O/disp2_s$srv -o pf --output-format csv -- \
      python3 bench.py --per-frame-only --steps 2 --server $srv --display pipelined --display-format r11g11b10f \
      --readback-depth 2 > $O/disp2_s$srv.log 2>&1 || { tail -5 $O/disp2_s$srv.log; exit 1; }
  grep per_frame_only $O/disp2_s$srv.log | cut -c1-200
done
