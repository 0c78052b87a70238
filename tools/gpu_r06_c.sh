set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_per_frame.py tests/test_gpu_server.py tests/test_gpu_check_exec.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06c_pytest.log 2>&1 || { tail -30 gpurun_out/r06c_pytest.log; exit 1; }
tail -1 gpurun_out/r06c_pytest.log
O=gpurun_out/emulate
for f in 0 64; do
  timeout -k 10 240 python bench.py --queue-fill $f --no-per-frame --no-cpu-baseline --no-framed --no-fast-bvh --steps 8 \
      > $O/c_n1_f$f.json 2> $O/c_n1_f$f.err || exit 1
  python3 -c "import json; r=json.loads(open('$O/c_n1_f$f.json').read().strip().splitlines()[-1]); print('N=1 fill=$f', round(r['value']))"
done
for fs in 0 32; do
  timeout -k 10 240 python bench.py --emulate-ranks 8 --queue-fill 4 --frame-split $fs --no-per-frame --no-cpu-baseline \
      --no-framed --no-fast-bvh --steps 8 > $O/c_n8_s$fs.json 2> $O/c_n8_s$fs.err || exit 1
  python3 -c "
import json; r=json.loads(open('$O/c_n8_s$fs.json').read().strip().splitlines()[-1]); s=r['strong_scaling']
print('N=8 fill=4 split=$fs weak %.0f strong %.0f frac %.3f' % (r['value'], s['value'], s['per_gpu_frac_of_weak']))"
done
