#!/bin/bash
# queue exit count without acquire/release: parity of the variant on the per-frame tests, then per-frame rates
set -u
mkdir -p gpurun_out
HALOGEN_LIB=variants/lib_dr.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_per_frame.py > gpurun_out/dr_tests.log 2>&1 || { tail -30 gpurun_out/dr_tests.log; exit 1; }
tail -3 gpurun_out/dr_tests.log
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_dr.txt 2>&1 | tail -20 || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_dr.jsonl
