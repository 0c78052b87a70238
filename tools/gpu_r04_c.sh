#!/bin/bash
# ray-sort experiment: parity of the HG_RAY_SORT builds (goldens + full-size C3 rows, streaming kernel), then the
# interleaved C3 / C3F / C2 sweep against the product build; the strict per-frame leg of the new 12-stream default
set -u
mkdir -p gpurun_out
for v in 1 2; do
  HALOGEN_LIB=variants/lib_rs$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider -m gpu -k "(stream and not C2 and not C5) or one_frame_launches" \
      tests/test_gpu_parity.py::test_gpu_matches_golden tests/test_gpu_parity.py::test_gpu_full_size_rows_match_oracle \
      tests/test_gpu_per_frame.py::test_gpu_one_frame_launches_match_golden > gpurun_out/pytest_rs$v.log 2>&1; rc=$?
  echo "rs$v parity rc=$rc"; tail -2 gpurun_out/pytest_rs$v.log; [ $rc -eq 0 ] || exit $rc
done
SWEEP_TIMEOUT=300 bash tools/sweep.sh tools/sweeps/sweep_r04_b.txt || exit $?
cat gpurun_out/sweep.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(round(r['value'],1), r['args'])"
for co in 1 32; do
  timeout -k 10 300 python bench.py --per-frame-only --steps 4 --coalesce $co > gpurun_out/pf_c_co$co.json 2>&1; rc=$?
  echo "perframe co=$co rc=$rc"; tail -1 gpurun_out/pf_c_co$co.json; [ $rc -eq 0 ] || exit $rc
done
