set -o pipefail
O=gpurun_out/emulate
mkdir -p $O gpurun_out/display
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
# display one frame behind (R11G11B10F) and strict, per-call launches: the shipped library and the drain-priority variant
for lib in shipped drainprio; do
  L=""; [ $lib = drainprio ] && L=$PWD/variants/drainprio/libhalogen_hip.so
  for mode in "--display pipelined --display-format r11g11b10f --readback-depth 2" "--display none"; do
    HALOGEN_LIB=$L timeout -k 10 240 python bench.py --per-frame-only --steps 4 --server 0 $mode > gpurun_out/display/$lib.json 2> gpurun_out/display/$lib.err || exit 1
    echo "$lib [$mode]: $(cut -c1-120 gpurun_out/display/$lib.json)"
  done
done
