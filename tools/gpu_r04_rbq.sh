#!/bin/bash
# per-frame display at display copy stream on its own queue
set -u
mkdir -p gpurun_out
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_rbq.txt 2>&1 | tail -20 || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_rbq.jsonl
