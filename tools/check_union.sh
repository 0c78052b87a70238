#!/bin/bash
# The roofline's launch basis (union of the trace launches' spans) from bench.py's HIP events against rocprofv3's trace.
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 8 > gpurun_out/b_union.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/u_stats -o stats --output-format csv -- \
    python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-framed --no-per-frame --no-counters > gpurun_out/prof/u_stats.log 2>&1 || exit $?
