#!/bin/bash
# A/B: the render server's XCD heads taking runs of B consecutive tiles (variants/libhalogen_run<B>.so, built with
# -DHG_SV_TILE_RUN=B) against the shipped library (B = HG_SV_TILE_RUN): the server tests on each variant, then strict / display at
# once / one frame behind, alternating libraries, one bench process per point under its own limit.  Build the variants
# here first (not on the box): for b in 1 4 16; do make -C halogen-pathtracer_amd OUT=$PWD/variants/libhalogen_run$b.so \
#   BUILD=$PWD/build_v_run$b EXTRA="-DHG_SV_TILE_RUN=${b}u"; done   (the shipped library is then B = HG_SV_TILE_RUN)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/server_runs
mkdir -p $O
for b in ${RUNS:-1 4 16}; do
  HALOGEN_LIB=$PWD/variants/libhalogen_run$b.so timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py -x -q \
      --timeout 240 --timeout-method thread > $O/tests_$b.log 2>&1 || { tail -30 $O/tests_$b.log; exit 1; }
  echo "run $b: $(tail -1 $O/tests_$b.log)"
done
for rep in 1 2; do
  for b in shipped ${RUNS:-1 4 16}; do
    for disp in none sync pipelined; do
      tag=b${b}_${disp}_${rep}
      if [ $b = shipped ]; then unset HALOGEN_LIB; else export HALOGEN_LIB=$PWD/variants/libhalogen_run$b.so; fi
      timeout -k 10 200 python bench.py --per-frame-only --server 2 --display $disp --display-format r11g11b10f \
          --launch-frames 1 --frames-per-step 64 --steps 8 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
      python3 -c "import json; r = json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(r['value']))"
    done
  done
done
