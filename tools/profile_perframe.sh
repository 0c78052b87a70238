#!/bin/bash
# rocprofv3 kernel trace + stats of the one-dispatch-per-frame operating point (bench.py --per-frame-only)
set -u
TAG=${TAG:-r03}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_perframe" -o pf --output-format csv -- \
    python3 bench.py --per-frame-only --steps 2 ${PF_ARGS:-} > "$OUT/${TAG}_perframe.log" 2>&1
rc=$?; echo "perframe rc=$rc"; tail -3 "$OUT/${TAG}_perframe.log"; exit $rc
