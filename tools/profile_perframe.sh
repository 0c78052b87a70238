#!/bin/bash
# rocprofv3 kernel trace + stats of the one-dispatch-per-frame operating point (bench.py --per-frame-only)
set -u
TAG=${TAG:-r04}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
# strict (every hg_render call its own: the render server, which the host's run-ahead engages), the same with the
# server off (a launch per call), and the default coalescing window
for run in co1 co1_srv0 co32; do
  case $run in co1) a="--coalesce 1";; co1_srv0) a="--coalesce 1 --server 0";; co32) a="--coalesce 32";; esac
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_perframe_$run" -o pf --output-format csv -- \
      python3 bench.py --per-frame-only --steps 2 $a ${PF_ARGS:-} > "$OUT/${TAG}_perframe_$run.log" 2>&1
  rc=$?; echo "perframe $run rc=$rc"; grep per_frame_only "$OUT/${TAG}_perframe_$run.log"; [ $rc -eq 0 ] || exit $rc
done
