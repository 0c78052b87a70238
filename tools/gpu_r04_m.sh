#!/bin/bash
# per-frame legs: 1-frame traces on the first idle stream vs in turn; a kernel + copy trace of the display at depth 2
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_depth.txt 2>&1 | tail -12 || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_depth.jsonl
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof/r04m_display2_pick -o pf \
    --output-format csv -- python3 bench.py --per-frame-only --steps 2 --coalesce 1 --display pipelined \
    --display-format r11g11b10f --readback-depth 2 --lane-pick 1 > gpurun_out/prof/r04m_display2_pick.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
