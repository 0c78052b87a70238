#!/bin/bash
# A/B of variant libraries: a parity subset of LIB (goldens, 1-frame launches, tile order, frame splits), then a sweep.
#   LIB=variants/lib_x.so SWEEP=tools/sweeps/sweep_r03_c.txt bash tools/gpu_ab_r03.sh
set -u
mkdir -p gpurun_out
if [ -n "${LIB:-}" ]; then
  HALOGEN_LIB=$LIB timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_per_frame.py tests/test_gpu_comm.py tests/test_gpu_fuzz.py -m gpu \
    -k "${PYTEST_K:-not dead_peer}" > gpurun_out/pt_ab.log 2>&1
  rc=$?; tail -4 gpurun_out/pt_ab.log; [ $rc -le 1 ] || exit $rc
fi
SWEEP_TIMEOUT=${SWEEP_TIMEOUT:-200} bash tools/sweep.sh "$SWEEP" 2>&1 | grep -v "^$" | tail -20
