#!/bin/bash
# Emulated strong shares against the frame split (per-tile waves, HG_OPT_QUEUE_FILL 0): SPLITS per N in "N:s1,s2" pairs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/split
mkdir -p $O
for spec in ${SPECS:-2:1,2 4:2,4 8:4,8}; do
  n=${spec%%:*}
  for fs in $(echo ${spec#*:} | tr ',' ' '); do
    timeout -k 10 200 python bench.py --emulate-ranks $n --queue-fill 0 --frame-split $fs --no-per-frame --no-cpu-baseline \
        --no-framed --no-fast-bvh --steps 8 > $O/n${n}_s$fs.json 2>/dev/null || exit 1
    python3 -c "import json; r=json.loads(open('$O/n${n}_s$fs.json').read().strip().splitlines()[-1]); print('N=$n split $fs strong', round(r['strong_scaling']['value']))"
  done
done
