#!/bin/bash
# Rank 0's share of an N-rank render on one GPU (--emulate-ranks): the weak line and the strong-scaling leg, N = 2, 4, 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05k
mkdir -p $O
for n in 2 4 8; do
  timeout -k 10 240 python -u bench.py --emulate-ranks $n --no-per-frame --no-cpu-baseline --no-framed --no-fast-bvh \
      > $O/emu$n.json 2> $O/emu$n.err || { tail -3 $O/emu$n.err; exit 1; }
  python3 -c "
import json; l = json.loads(open('$O/emu$n.json').read().strip().splitlines()[-1]); s = l['strong_scaling']
print('N=$n weak', round(l['value'], 1), 'ms/step', round(l['ms_per_step'], 2), '| strong share', round(s['value'], 1),
      'if balanced', round(s.get('value_if_balanced', 0), 1), 'ms/step', round(s['ms_per_step'], 2), 'tiles', s['per_rank'][0]['tiles'])"
done
