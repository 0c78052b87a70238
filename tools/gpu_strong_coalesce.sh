#!/bin/bash
# Strong shares (bench.py --emulate-ranks N) with the strong leg's calls held for one launch (HG_OPT_COALESCE) and the
# queue form on or off: one bench process per point, each under its own limit.  POINTS: "N:fill:coalesce ..."
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/strong_coalesce
mkdir -p $O
for pt in ${POINTS:-8:-1:-1 8:0:512 8:-1:512 8:0:1024 4:-1:-1 4:0:256 4:0:512}; do
  IFS=: read n f k <<< "$pt"
  tag=n${n}_f${f}_k${k}
  timeout -k 10 240 python bench.py --emulate-ranks $n --queue-fill $f --strong-coalesce $k --no-per-frame \
      --no-cpu-baseline --no-framed --no-fast-bvh --steps ${STEPS:-16} > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; r = json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); s = r['strong_scaling']
print('N=$n fill=$f coalesce=$k weak %.0f strong %.0f (%.3f) ms/step %.3f' % (r['value'], s['value'], s['value'] / r['value'], s['ms_per_step']))"
done
