#!/bin/bash
# deep PMC of the ray-sort build against the product build (C3 timed launches only), and a kernel + memory-copy trace
# of the pipelined R11G11B10 display at depth 8
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
export BENCH_ARGS="--steps 4 --warmup 1 --no-cpu-baseline --no-framed --no-per-frame"
TAG=r04f_base bash tools/pmc_deep.sh || exit $?
HALOGEN_LIB=variants/lib_rs1.so TAG=r04f_rs1 bash tools/pmc_deep.sh || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof/r04f_display8 -o pf \
    --output-format csv -- python3 bench.py --per-frame-only --steps 2 --coalesce 1 --display pipelined \
    --display-format r11g11b10f --readback-depth 8 > gpurun_out/prof_r04f_display8.log 2>&1; rc=$?
echo "prof display8 rc=$rc"; grep per_frame_only gpurun_out/prof_r04f_display8.log
exit $rc
