#!/bin/bash
# path migration A/B: parity of the variant on the per-frame tests, then strict per-frame rates
set -u
mkdir -p gpurun_out
HALOGEN_LIB=variants/lib_mig_k1i48.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_per_frame.py > gpurun_out/mig_tests.log 2>&1 || { tail -30 gpurun_out/mig_tests.log; exit 1; }
tail -3 gpurun_out/mig_tests.log
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_mig.txt 2>&1 | tail -20 || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_mig.jsonl
