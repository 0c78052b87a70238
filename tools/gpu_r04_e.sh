#!/bin/bash
# display path after the one-wave untile: sweep + rocprof kernel trace of the pipelined R11G11B10 leg; deep PMC of the
# ray-sort build against the product build (C3)
set -u
mkdir -p gpurun_out/prof
bash tools/pf_sweep.sh tools/sweeps/sweep_r04_c.txt || exit $?
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/r04e_display -o pf --output-format csv -- \
    python3 bench.py --per-frame-only --steps 2 --coalesce 1 --display pipelined --display-format r11g11b10f \
    > gpurun_out/prof_r04e_display.log 2>&1; rc=$?
echo "prof display rc=$rc"; grep per_frame_only gpurun_out/prof_r04e_display.log; [ $rc -eq 0 ] || exit $rc
TAG=r04e_base bash tools/pmc_deep.sh || exit $?
HALOGEN_LIB=variants/lib_rs1.so TAG=r04e_rs1 bash tools/pmc_deep.sh || exit $?
