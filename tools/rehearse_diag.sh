set -u
mkdir -p gpurun_out/dist
export HALOGEN_BENCH_DEVICE=0
ARGS="--config C3 --width 640 --height 360 --steps 1 --warmup 1 --no-cpu-baseline --frames-per-step 8"
for K in stream regen; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --dist-backend gloo $ARGS --kernel $K --save-image gpurun_out/dist/n2_$K.npy > gpurun_out/dist/n2_$K.json 2> gpurun_out/dist/n2_$K.err || exit 1
  timeout -k 10 300 python bench.py $ARGS --kernel $K --frames-per-step 16 --save-image gpurun_out/dist/n1_$K.npy > gpurun_out/dist/n1_$K.json 2> gpurun_out/dist/n1_$K.err || exit 1
  timeout -k 10 300 python bench.py $ARGS --kernel $K --frames-per-step 16 --no-counters --save-image gpurun_out/dist/n1nc_$K.npy > /dev/null 2>&1 || exit 1
done
python - <<'PY'
import numpy as np
d='gpurun_out/dist/'
for K in ('stream','regen'):
    a=np.load(d+f'n2_{K}.npy'); b=np.load(d+f'n1_{K}.npy'); c=np.load(d+f'n1nc_{K}.npy')
    diff=(a.view(np.uint32)!=b.view(np.uint32)).any(-1)
    print(K, 'n2 vs n1 differing px:', int(diff.sum()), ' n1 vs n1(no counters):', int((b.view(np.uint32)!=c.view(np.uint32)).any(-1).sum()))
    if diff.any():
        ys,xs=np.nonzero(diff); print('  first', list(zip(ys[:5],xs[:5])), 'tiles', sorted(set(((y//8)*80+x//8) for y,x in zip(ys,xs)))[:10])
a=np.load(d+'n1_stream.npy'); b=np.load(d+'n1_regen.npy')
print('n1 stream vs regen:', int((a.view(np.uint32)!=b.view(np.uint32)).any(-1).sum()))
PY
