#!/bin/bash
# final round-4 library, part 2: the C2 / C5 profile passes and the bench line
set -u
mkdir -p gpurun_out
TAG=${TAG:-r04a} CONFIGS="C2 C5" bash tools/profile_r04.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err; rc=$?
echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_h.json; tail -3 gpurun_out/bench_h.err
exit $rc
