#!/bin/bash
# the whole -m gpu suite on the in-tree library, then an A/B sweep (sweep file $1)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error|FAILED" gpurun_out/pytest_gpu.log | tail -6
[ $rc -le 1 ] || exit $rc
SWEEP_TIMEOUT=200 bash tools/sweep.sh "$1" 2>&1 | grep -v "^$" | tail -20
