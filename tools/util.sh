set -u
# counters + SIMD utilisation + traversal/shading clock split per config (one bench process per config)
for c in C3 C2 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/util_$c.json 2> gpurun_out/util_$c.err || exit $?
  python3 -c "import json; r=json.load(open('gpurun_out/util_$c.json')); print('$c', round(r['value']), r['simd_utilisation'], r['phase_split'], r['counters_per_path'])"
done
