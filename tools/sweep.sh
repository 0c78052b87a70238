#!/bin/bash
# Configuration sweep of bench.py, one process per line.  A line is "[VAR=value ...] bench-args"; VAR=value
# words (e.g. HALOGEN_LIB=variants/lib_w8.so) become the environment of that run.  Stops on a fault/timeout.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/sweep.jsonl
: > $OUT
while read -r line; do
  [ -z "$line" ] && continue
  envs=(); args=()
  for w in $line; do
    if [[ "$w" == *=* && "$w" != --* ]]; then envs+=("$w"); else args+=("$w"); fi
  done
  env "${envs[@]}" timeout -k 10 ${SWEEP_TIMEOUT:-300} python bench.py --no-cpu-baseline "${args[@]}" > gpurun_out/sweep_one.json 2> gpurun_out/sweep_one.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $line"; tail -5 gpurun_out/sweep_one.err; exit $rc; fi
  python3 -c "
import json,sys; r=json.loads(open('gpurun_out/sweep_one.json').read().strip().splitlines()[-1])
r['args']='$line'; print(json.dumps(r))
k=r.get('kernel_ms',{})
tr=(k.get('trace_total',0)/max(k.get('trace_launches',1),1))
print(f\"{r['value']:9.1f} Mpaths/s {r['ms_per_step']:9.3f} ms/step trace_total={k.get('trace_total',0):8.1f}ms  $line\", file=sys.stderr)" >> $OUT
done < "${1:-/dev/stdin}"
