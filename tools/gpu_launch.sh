#!/bin/bash
# bench.py --gpus N without a launcher on the one-GPU box (every rank on device 0, gloo): the parent starts the ranks,
# relays rank 0's line; the gathered weak image must equal one context's N*F frames, the strong one one context's image.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/launch
mkdir -p $O
ARGS="--config C3 --width 640 --height 360 --steps 1 --warmup 1 --no-cpu-baseline --frames-per-step 8 --gather torch --no-abi-check"
HALOGEN_BENCH_DEVICE=0 timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo $ARGS --save-image $O/img_n2.npy \
    > $O/n2.json 2> $O/n2.err || { echo "self-launched N=2 failed"; tail -20 $O/n2.err; exit 1; }
echo "lines on stdout: $(grep -c '^{' $O/n2.json)"
timeout -k 10 300 python3 bench.py $ARGS --frames-per-step 16 --save-image $O/img_1x2.npy > $O/1x2.json 2> $O/1x2.err || exit 1
python3 -c "
import json, numpy as np
a = np.load('$O/img_n2.npy'); b = np.load('$O/img_1x2.npy')
r = json.loads(open('$O/n2.json').read().strip().splitlines()[-1]); st = r['strong_scaling']
print('self-launched N=2: n_gpus', r['n_gpus'], 'weak gathered == 1-rank 16 frames:', np.array_equal(a.view(np.uint32), b.view(np.uint32)),
      '| strong gathered == one context:', st.get('gathered_bit_identical_to_one_context'))"
