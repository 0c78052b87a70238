set -o pipefail
mkdir -p gpurun_out/display
timeout -k 10 900 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_display.py tests/test_host_cpp.py tests/test_gpu_per_frame.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06h_pytest.log 2>&1 || { tail -40 gpurun_out/r06h_pytest.log; exit 1; }
tail -1 gpurun_out/r06h_pytest.log
for ahead in 4 8 14; do
  for depth in 1 2; do
    mode="--display pipelined"; [ $depth = 1 ] && mode="--display sync"
    timeout -k 10 240 python bench.py --per-frame-only --steps 4 --server-ahead $ahead $mode --display-format r11g11b10f \
        --readback-depth $depth > gpurun_out/display/h_a${ahead}_d$depth.json 2> gpurun_out/display/h_a${ahead}_d$depth.err || { tail -5 gpurun_out/display/h_a${ahead}_d$depth.err; exit 1; }
    python3 -c "
import json; r=json.loads(open('gpurun_out/display/h_a${ahead}_d$depth.json').read())
print('ahead $ahead depth $depth: %.0f Mpaths/s (%.3f of 3490)' % (r['value'], r['value']/3490))"
  done
done
