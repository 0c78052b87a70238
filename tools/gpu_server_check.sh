#!/bin/bash
# The render server's tests, then its strict and display-at-once points (one bench process each, own limits)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/server_check
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_display.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for disp in none sync pipelined; do
  timeout -k 10 200 python bench.py --per-frame-only --server 2 --display $disp --display-format r11g11b10f --launch-frames 1 \
      --frames-per-step 64 --steps 8 --no-cpu-baseline > $O/$disp.json 2> $O/$disp.err || { tail -5 $O/$disp.err; exit 1; }
  python3 -c "import json; r = json.loads(open('$O/$disp.json').read().strip().splitlines()[-1]); print('$disp', round(r['value']))"
done
