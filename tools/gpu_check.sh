#!/bin/bash
# One GPU session: smoke, gpu tests, short bench.  Every GPU step has its own time limit; a fault / abort /
# timeout (exit >= 124 or 134/139) stops the script; an ordinary test failure (exit 1) does not.
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc
