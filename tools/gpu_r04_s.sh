#!/bin/bash
# wave-deduplicated node fetch (HG_NODE_DEDUP variant): parity on the variant library, then an interleaved A/B
set -u
mkdir -p gpurun_out
HALOGEN_LIB=variants/lib_dedup.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_gpu_per_frame.py tests/test_gpu_fuzz.py \
    > gpurun_out/pytest_s.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_s.log; [ $rc -eq 0 ] || exit $rc
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_dedup.txt 2>&1 | tail -12 || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_dedup.jsonl
