set -o pipefail
mkdir -p gpurun_out/display gpurun_out/emulate
timeout -k 10 600 python -u -m pytest tests/test_gpu_display.py tests/test_gpu_server.py tests/test_gpu_parity.py tests/test_gpu_per_frame.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06f_pytest.log 2>&1 || { tail -30 gpurun_out/r06f_pytest.log; exit 1; }
tail -1 gpurun_out/r06f_pytest.log
for side in 0 2; do
  for depth in 1 2 4; do
    mode="--display pipelined"; [ $depth = 1 ] && mode="--display sync"
    timeout -k 10 240 python bench.py --per-frame-only --steps 4 --server 0 $mode --display-format r11g11b10f --readback-depth $depth \
        --readback-stream $side > gpurun_out/display/s${side}_d$depth.json 2> gpurun_out/display/s${side}_d$depth.err || exit 1
    echo "side $side depth $depth: $(cut -c1-100 gpurun_out/display/s${side}_d$depth.json)"
  done
done
for n in 4 8; do
  timeout -k 10 240 python bench.py --emulate-ranks $n --no-per-frame --no-cpu-baseline --no-framed --no-fast-bvh --steps 8 \
      > gpurun_out/emulate/f_n$n.json 2> gpurun_out/emulate/f_n$n.err || exit 1
  python3 -c "
import json; r=json.loads(open('gpurun_out/emulate/f_n$n.json').read().strip().splitlines()[-1]); s=r['strong_scaling']
print('N=$n default: weak %.0f strong %.0f' % (r['value'], s['value']))"
done
