#!/bin/bash
# Multi-tile streaming waves (HG_OPT_WAVE_UNITS): parity tests, then the A/B sweep
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_wave_units.py tests/test_gpu_parity.py > gpurun_out/pytest_j.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_j.log; [ $rc -eq 0 ] || exit $rc
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_wu.txt 2>&1 | tail -20
