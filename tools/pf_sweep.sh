#!/bin/bash
# Per-frame sweep: one bench.py --per-frame-only process per line ("[VAR=value ...] bench-args"); each line's JSON is
# appended (with its args) to gpurun_out/pf_sweep.jsonl.  Stops on a fault / timeout.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/pf_sweep.jsonl
: > $OUT
while read -r line; do
  [ -z "$line" ] && continue
  envs=(); args=()
  for w in $line; do
    if [[ "$w" == *=* && "$w" != --* ]]; then envs+=("$w"); else args+=("$w"); fi
  done
  env "${envs[@]}" timeout -k 10 ${SWEEP_TIMEOUT:-200} python bench.py "${args[@]}" > gpurun_out/pf_one.json 2> gpurun_out/pf_one.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $line"; tail -5 gpurun_out/pf_one.err; exit $rc; fi
  python3 -c "
import json; r=json.loads(open('gpurun_out/pf_one.json').read().strip().splitlines()[-1]); r['args']='$line'
print(json.dumps(r))" >> $OUT
  tail -1 $OUT | cut -c1-200
done < "${1:-/dev/stdin}"
