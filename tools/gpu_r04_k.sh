#!/bin/bash
# frame-split sweep (shorter waves), then kernel + memory-copy traces of the per-frame legs: strict without display,
# pipelined R11G11B10F display at depth 2 (one frame behind) and 8
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_split.txt 2>&1 | tail -8 || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_split.jsonl
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof/$tag -o pf \
      --output-format csv -- python3 bench.py --per-frame-only --steps 2 --coalesce 1 "$@" > gpurun_out/prof/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; grep per_frame_only gpurun_out/prof/$tag.log | cut -c1-300; return $rc
}
run r04k_strict || exit $?
run r04k_display2 --display pipelined --display-format r11g11b10f --readback-depth 2 || exit $?
run r04k_display8 --display pipelined --display-format r11g11b10f --readback-depth 8 || exit $?
