set -u
# shading sub-phase clock split of the streaming kernel (analysis builds with HG_PHASE_DETAIL=1 / 2)
for v in ${PHASES:-phase phase2 phase3}; do
  timeout -k 10 300 env HALOGEN_LIB=variants/lib_$v.so python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${v}_C3.json 2> gpurun_out/${v}_C3.err || exit $?
  python3 -c "import json; r=json.load(open('gpurun_out/${v}_C3.json')); print('$v', round(r['value']), r['phase_split'], r['shading_detail'])"
done
