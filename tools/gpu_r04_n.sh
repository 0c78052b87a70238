#!/bin/bash
# per-frame display at readback depths 2..16, 1-frame traces on the first idle stream vs in turn; strict
set -u
mkdir -p gpurun_out
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_depth.txt 2>&1 | tail -20 || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_depth.jsonl
