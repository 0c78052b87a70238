#!/bin/bash
# display-format tests (Python, C++ host, comm), then the lanes x divisor sweep of strict per-frame launches
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 120 tools/micro_lane_order > gpurun_out/micro_lane_order.json; rc=$?
echo "micro_lane_order rc=$rc"; cat gpurun_out/micro_lane_order.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_display.py "tests/test_gpu_comm.py::test_gpu_comm_display_readback_pipelined" \
    "tests/test_host_cpp.py::test_gpu_cpp_pipelined_display_matches_golden" tests/test_gpu_upload.py \
    > gpurun_out/pytest_b.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_b.log | tail -5
ok $rc || exit $rc
bash tools/pf_sweep.sh tools/sweeps/sweep_r04_a.txt || exit $?
timeout -k 10 600 python bench.py --steps 8 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err; rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_b.json; tail -3 gpurun_out/bench_b.err
exit $rc
