#!/bin/bash
# Round 4 library: smoke, the whole -m gpu suite, a bench line.  A fault / abort / timeout stops the script.
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -5
ok $rc || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err; rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_d.json; tail -3 gpurun_out/bench_d.err
exit $rc
