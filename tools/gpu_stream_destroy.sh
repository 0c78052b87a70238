#!/bin/bash
# tools/micro_stream_destroy: one case per process, each under its own time limit; the first case that times out (a
# hung hipStreamDestroy) ends the call (no GPU step after a kill).  CASES overrides the list (';'-separated).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/stream_destroy
mkdir -p $O
IFS=';' read -ra LIST <<< "${CASES:-masked_last server 1 1;masked_first none 0 0;masked_first trivial 0 0;masked_first server 0 0;masked_first server 1 0;masked_first server 1 1}"
for c in "${LIST[@]}"; do
  n=$(echo $c | tr ' ' '_')
  timeout -k 5 30 ./tools/micro_stream_destroy $c > $O/$n.out 2> $O/$n.err; rc=$?
  echo "case [$c] rc=$rc: $(tail -1 $O/$n.err)"
  [ $rc -eq 0 ] || { tail -6 $O/$n.err; exit $rc; }
done
