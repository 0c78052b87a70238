#!/bin/bash
# Render-server diagnostics: 200 frames k per call against the batched launch, short gate timeout, progress logged.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05b
mkdir -p $O
export HALOGEN_SERVER_GATE_TIMEOUT_MS=1500
HALOGEN_SERVER_TRACE=1 timeout -k 10 60 python3 -u tools/server_diag.py $O/diag_pc1.log --frames 200 --per-call 1 \
    --tilings none 2> $O/diag_pc1.err; rc=$?; echo "pc1 rc=$rc"; cat $O/diag_pc1.log; tail -c 3000 $O/diag_pc1.err
[ $rc -eq 0 ] || exit $rc
true
