set -o pipefail
O=gpurun_out/emulate
mkdir -p $O
# the queue form's per-item cost at N=1 (every C3 launch through the queue) against the per-tile waves
for f in 0 64; do
  timeout -k 10 240 python bench.py --queue-fill $f --no-per-frame --no-cpu-baseline --no-framed --no-fast-bvh --steps 8 \
      > $O/n1_f$f.json 2> $O/n1_f$f.err || exit 1
  python3 -c "import json; r=json.loads(open('$O/n1_f$f.json').read().strip().splitlines()[-1]); print('N=1 fill=$f', round(r['value']))"
done
# smaller queue units / more per-tile waves at N=8
for fs in 16 32; do
  for f in 0 4; do
    timeout -k 10 240 python bench.py --emulate-ranks 8 --queue-fill $f --frame-split $fs --no-per-frame --no-cpu-baseline \
        --no-framed --no-fast-bvh --steps 8 > $O/n8_f${f}_s$fs.json 2> $O/n8_f${f}_s$fs.err || exit 1
    python3 -c "
import json; r=json.loads(open('$O/n8_f${f}_s$fs.json').read().strip().splitlines()[-1]); s=r['strong_scaling']
print('N=8 fill=$f split=$fs weak %.0f strong %.0f frac %.3f' % (r['value'], s['value'], s['per_gpu_frac_of_weak']))"
  done
done
CASES="r05pre_trace HG_TD_DEFER_HOST=1;r05pre_trace HG_TD_DEFER_EVENTS=1;r05pre_trace HG_TD_DEFER_BUFS=1" bash tools/gpu_teardown_r05pre.sh
