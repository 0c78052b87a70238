#!/bin/bash
# A/B session: parity of one variant library (the whole -m gpu suite against it), then a bench sweep.
#   LIB=variants/lib_x.so SWEEP=tools/sweepNN.txt bash tools/ab.sh
set -u
mkdir -p gpurun_out
if [ -n "${LIB:-}" ]; then
  HALOGEN_LIB=$LIB timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pt_ab.log 2>&1
  rc=$?; tail -4 gpurun_out/pt_ab.log; [ $rc -le 1 ] || exit $rc
fi
SWEEP_TIMEOUT=${SWEEP_TIMEOUT:-200} bash tools/sweep.sh "$SWEEP" || exit $?
python3 - <<'PY'
import json
for l in open("gpurun_out/sweep.jsonl"):
    r = json.loads(l)
    print(f"{r['value']:8.1f} {r.get('simd_utilisation')} {r['args']}")
PY
