#!/bin/bash
# A/B of render-server variant libraries against the shipped one: for each name in VARIANTS, variants/libhalogen_<name>.so
# (built here first, not on the box, e.g. make -C halogen-pathtracer_amd OUT=$PWD/variants/libhalogen_claim8.so
# BUILD=$PWD/build_v_claim8 EXTRA="-DHG_SV_CLAIM=8u"): the server tests on each variant, then strict / display at once /
# one frame behind (C3, server forced, 8 x 64 one-frame calls, R11G11B10F), alternating libraries over two rounds, one
# bench process per point under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/server_ab
mkdir -p $O
for v in ${VARIANTS:?set VARIANTS}; do
  HALOGEN_LIB=$PWD/variants/libhalogen_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py -x -q \
      --timeout 240 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
for rep in 1 2; do
  for v in shipped $VARIANTS; do
    for disp in none sync pipelined; do
      tag=${v}_${disp}_${rep}
      if [ $v = shipped ]; then unset HALOGEN_LIB; else export HALOGEN_LIB=$PWD/variants/libhalogen_$v.so; fi
      timeout -k 10 200 python bench.py --per-frame-only --server 2 --display $disp --display-format r11g11b10f \
          --launch-frames 1 --frames-per-step 64 --steps 8 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
      python3 -c "import json; r = json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(r['value']))"
    done
  done
done
