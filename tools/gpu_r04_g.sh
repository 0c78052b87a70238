#!/bin/bash
# final round-4 library, part 1: the upload tests, the C3 / C3F profile passes (stats + PMC incl. VMEM instruction
# counts) and the per-frame profile
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_upload.py tests/test_gpu_display.py > gpurun_out/pytest_g.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_g.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r04a} CONFIGS="C3 C3F" bash tools/profile_r04.sh || exit $?
TAG=${TAG:-r04a} bash tools/profile_perframe.sh || exit $?
