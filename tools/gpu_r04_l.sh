#!/bin/bash
# per-frame legs with host time per call, readback waits blocking vs polling
set -u
mkdir -p gpurun_out
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r04_host.txt 2>&1 | tail -12 || exit $?
python3 -c "
import json
for l in open('gpurun_out/sweep.jsonl'):
    r=json.loads(l); print(round(r['value'],1), {k: round(v,4) for k,v in r['host_ms_per_call'].items()}, r['args'][36:])
"
