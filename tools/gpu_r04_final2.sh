#!/bin/bash
# final round-4 library, part 2: C2 / C5 profile passes and the per-frame profile
set -u
mkdir -p gpurun_out
TAG=${TAG:-r04x} CONFIGS="C2 C5" bash tools/profile_r04.sh || exit $?
TAG=${TAG:-r04x} bash tools/profile_perframe.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_final3.json 2> gpurun_out/bench_final3.err; rc=$?
echo "bench rc=$rc"; tail -c 200 gpurun_out/bench_final3.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_final3.err; exit $rc; }
