#!/bin/bash
# Round-3 session: queue variant parity + A/B sweep, then WRITE_SIZE passes (default tree, no frame colours, 24-entry
# LDS stack) for the write-traffic attribution.
set -u
LIB=variants/lib_qF.so SWEEP=tools/sweeps/sweep_r03_d.txt bash tools/gpu_ab_r03.sh || exit $?
bash tools/pmc_write_ab.sh nofc stk24 || exit $?
for v in default nofc stk24; do echo "== $v"; python3 tools/pmc_table.py gpurun_out/pmcw/$v; done
