#!/bin/bash
# Strong-scaling shares on one GPU: bench.py --emulate-ranks N (rank 0's 1/N of the tiles; the weak line and the strong
# leg), for each N in $RANKS and each HG_OPT_QUEUE_FILL in $FILLS.  One bench process per point, each under its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/emulate
mkdir -p $O
for n in ${RANKS:-2 4 8}; do
  for f in ${FILLS:-0 4}; do
    timeout -k 10 240 python bench.py --emulate-ranks $n --queue-fill $f --no-per-frame --no-cpu-baseline --no-framed \
        --no-fast-bvh --steps ${STEPS:-8} ${EXTRA:-} > $O/n${n}_f${f}.json 2> $O/n${n}_f${f}.err || { tail -5 $O/n${n}_f${f}.err; exit 1; }
    python3 -c "
import json; r = json.loads(open('$O/n${n}_f${f}.json').read().strip().splitlines()[-1]); s = r['strong_scaling']
print('N=$n fill=$f weak %.0f strong %.0f ms/step %.3f' % (r['value'], s['value'], s['ms_per_step']))"
  done
done
