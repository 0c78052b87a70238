#!/bin/bash
# The render server's unit order: the cost order (default) against raster order (HG_OPT_TILE_ORDER 0), strict per-frame
# C3 (512 1-frame calls, the server forced) and the display at once, one bench process per point under its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/server_order
mkdir -p $O
for rep in 1 2; do
  for to in 1 0; do
    for disp in none sync; do
      tag=to${to}_${disp}_${rep}
      timeout -k 10 200 python bench.py --per-frame-only --server 2 --tile-order $to --display $disp \
          --display-format r11g11b10f --launch-frames 1 --frames-per-step 64 --steps 8 --no-cpu-baseline \
          > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
      python3 -c "import json; r = json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(r['value']))"
    done
  done
done
