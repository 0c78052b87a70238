#!/bin/bash
# Round 4, first check of the per-frame changes: smoke, the per-frame / order / chunk-tail / check-build tests, the
# strict and coalesced per-frame legs, and a rocprof kernel trace of the strict leg.
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_per_frame.py tests/test_gpu_display.py tests/test_gpu_regen_noitems.py tests/test_gpu_check_exec.py \
    "tests/test_gpu_comm.py::test_gpu_comm_display_readback_pipelined" \
    "tests/test_gpu_parity.py::test_gpu_tile_order_bit_exact" > gpurun_out/pytest_a.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_a.log | tail -5
ok $rc || exit $rc
for co in 1 32; do
  timeout -k 10 300 python bench.py --per-frame-only --steps 4 --coalesce $co > gpurun_out/pf_co$co.json 2>&1; rc=$?
  echo "perframe co=$co rc=$rc"; tail -2 gpurun_out/pf_co$co.json; [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/r04a_perframe_co1 -o pf --output-format csv -- \
    python3 bench.py --per-frame-only --steps 2 --coalesce 1 > gpurun_out/prof_r04a.log 2>&1; rc=$?
echo "prof rc=$rc"; grep per_frame_only gpurun_out/prof_r04a.log
exit $rc
