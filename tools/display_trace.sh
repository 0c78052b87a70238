#!/bin/bash
# Kernel + copy timeline of the R11G11B10F display one frame behind, a launch per call (server off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${DT_DIR:-display}
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $O/disp2_s${SRV:-0} -o pf --output-format csv -- \
    python3 bench.py --per-frame-only --steps 2 --server ${SRV:-0} --display pipelined --display-format r11g11b10f \
    --readback-depth 2 > $O/disp2_s${SRV:-0}.log 2>&1 || { tail -5 $O/disp2_s${SRV:-0}.log; exit 1; }
grep per_frame_only $O/disp2_s${SRV:-0}.log | cut -c1-200
ls $O/disp2_s${SRV:-0}
