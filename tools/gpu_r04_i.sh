#!/bin/bash
# Round 4 (re-entry): the whole GPU suite, the smoke, the bench line and the C3 / C3F profile passes of the current
# library.  Each GPU step has its own time limit; any failure ends the script.
set -u
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_i.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests \
    > gpurun_out/pytest_i.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_i.json 2> gpurun_out/bench_i.err; rc=$?
echo "bench rc=$rc"; tail -c 300 gpurun_out/bench_i.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_i.err; exit $rc; }
TAG=${TAG:-r04i} CONFIGS="C3 C3F" bash tools/profile_r04.sh || exit $?
