#!/bin/bash
# round-5 library, part 2: C2 / C5 profile passes, C3 on the SAH tree, and the bench line
set -u
mkdir -p gpurun_out
TAG=${TAG:-r05x} CONFIGS="C2 C5" bash tools/profile_r04.sh || exit $?
TAG=${TAG:-r05x}_sah CONFIGS="C3" BENCH_EXTRA="--bvh sah" bash tools/profile_r04.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_r05x.json 2> gpurun_out/bench_r05x.err; rc=$?
echo "bench rc=$rc"; tail -c 300 gpurun_out/bench_r05x.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_r05x.err; exit $rc; }
