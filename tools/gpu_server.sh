#!/bin/bash
# The render-server tests alone (handshake, lost frames, restarts), verbose, with the server trace of refusals counted
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/server
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_server.py -x -v -s --timeout 240 --timeout-method thread "$@" > $O/server.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|refused|passed|failed" $O/server.log | tail -40; exit $rc
