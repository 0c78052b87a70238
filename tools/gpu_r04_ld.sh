#!/bin/bash
# per-frame display at leaf-distribution threshold on SAH trees
set -u
mkdir -p gpurun_out
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_ld.txt 2>&1 | tail -20 || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_ld.jsonl
