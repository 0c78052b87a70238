#!/bin/bash
# the SAH-hierarchy GPU tests, then the full bench line (with the fast_bvh leg)
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_fast_bvh.py > gpurun_out/pytest_v.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_v.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/bench_v.json 2> gpurun_out/bench_v.err; rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_v.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_v.err; exit $rc; }
