#!/bin/bash
# the whole GPU suite on the current library, then quick C3 / C2 / strict checks of the deep-BLAS thresholds
set -u
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_z.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_z.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
    > gpurun_out/pytest_z.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_z.log; [ $rc -eq 0 ] || exit $rc
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_deep.txt 2>&1 | tail -8 || exit $?
