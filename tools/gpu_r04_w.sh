#!/bin/bash
# per-frame display at drain priority A/B
set -u
mkdir -p gpurun_out
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_dp.txt 2>&1 | tail -20 || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_dp.jsonl
