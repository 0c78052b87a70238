#!/bin/bash
# smoke + -m gpu suite + bench line (tools/gpu_r03.sh), then the trace-lane / HW-queue sweep (sweep_r03_t)
set -u
bash tools/gpu_r03.sh || exit $?
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r03_t.txt 2>&1 | grep -v "^$" | tail -20
