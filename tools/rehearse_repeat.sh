#!/bin/bash
# Repeat the 2-rank rehearsal (default kernel) and report differing tiles per repetition.
set -u
mkdir -p gpurun_out/dist
export HALOGEN_BENCH_DEVICE=0
ARGS="--config C3 --width 640 --height 360 --steps 1 --warmup 1 --no-cpu-baseline --frames-per-step 8"
timeout -k 10 200 python bench.py $ARGS --frames-per-step 16 --save-image gpurun_out/dist/ref1.npy > /dev/null 2>&1 || exit 1
for i in 1 2 3 4; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29520 + i)) bench.py --gpus 2 --dist-backend gloo $ARGS --save-image gpurun_out/dist/rep$i.npy \
      > gpurun_out/dist/rep$i.json 2> gpurun_out/dist/rep$i.err || exit 1
  python -c "
import numpy as np
a=np.load('gpurun_out/dist/rep$i.npy'); b=np.load('gpurun_out/dist/ref1.npy')
d=(a.view(np.uint32)!=b.view(np.uint32)).any(-1); z=(a[...,3]==0)
print('rep $i: differing px', int(d.sum()), 'alpha-0 px', int(z.sum()))"
done
