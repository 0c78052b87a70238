#!/bin/bash
# Teardown soak on the shipped library: N processes in a row, each a 200-frame
# render-server run of one-frame calls then hg_destroy (tools/server_diag.py), each under its own limit; a destroy that
# hangs is a host-side wait that the limit ends, and ends the script.  Prints each run's close time.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/teardown_soak
mkdir -p $O
export HALOGEN_SERVER_GATE_TIMEOUT_MS=3000
for i in $(seq 1 ${N:-40}); do
  timeout -k 5 60 python3 -u tools/server_diag.py $O/run$i.log --frames 200 --per-call 1 --tilings none \
      > $O/run$i.out 2> $O/run$i.err; rc=$?
  echo "run $i rc=$rc: $(grep "first bad" $O/run$i.log | tail -1) | $(tail -2 $O/run$i.log | tr "\n" " ")"
  [ $rc -eq 0 ] || exit $rc
done
