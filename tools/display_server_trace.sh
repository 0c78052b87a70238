#!/bin/bash
# Kernel + copy timeline of a per-frame R11G11B10F display through the render server: at once and one frame behind,
# tracing ahead (the default) and not (HG_OPT_SERVER_AHEAD 0, the server forced); tools/display_server_timeline.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/dst
mkdir -p $O
for c in "sync 1 4 1" "pipelined 2 4 1" "sync 1 0 2" "pipelined 2 0 2"; do
  set -- $c
  n=${1}_d${2}_a${3}
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $O/$n -o pf --output-format csv -- \
      python3 bench.py --per-frame-only --steps 2 --display $1 --display-format r11g11b10f --readback-depth $2 \
      --server-ahead $3 --server $4 > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "== $n: $(grep -o '"value": [0-9.]*' $O/$n.log | head -1)"
  python3 tools/display_server_timeline.py $O/$n 96
done
