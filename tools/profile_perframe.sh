#!/bin/bash
# rocprofv3 kernel trace + stats of the one-dispatch-per-frame operating point (bench.py --per-frame-only)
set -u
TAG=${TAG:-r04}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
for co in 1 32; do  # strict (every hg_render call its own launch) and the default coalescing window
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_perframe_co$co" -o pf --output-format csv -- \
      python3 bench.py --per-frame-only --steps 2 --coalesce $co ${PF_ARGS:-} > "$OUT/${TAG}_perframe_co$co.log" 2>&1
  rc=$?; echo "perframe coalesce $co rc=$rc"; grep per_frame_only "$OUT/${TAG}_perframe_co$co.log"; [ $rc -eq 0 ] || exit $rc
done
