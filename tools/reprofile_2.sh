#!/bin/bash
# After a library change, part 2 (tools/reprofile_after_library_change.md): C2 / C5 profile passes, C3 on the SAH tree, and the bench line
set -u
mkdir -p gpurun_out
TAG=${TAG:?set TAG} CONFIGS="C2 C5" bash tools/profile_r04.sh || exit $?
TAG=${TAG:?set TAG}_sah CONFIGS="C3" BENCH_EXTRA="--bvh sah" bash tools/profile_r04.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; rc=$?
echo "bench rc=$rc"; tail -c 300 gpurun_out/bench_${TAG}.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_${TAG}.err; exit $rc; }
