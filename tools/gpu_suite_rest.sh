#!/bin/bash
# The -m gpu suite from tests/test_gpu_upload.py on (the part after the last run's stop)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/suite
mkdir -p $O
files=$(ls tests/test_gpu_*.py | sort | awk '$0 >= "tests/test_gpu_upload.py"')
timeout -k 10 1000 python -u -m pytest $files -m gpu -x -v --timeout 240 --timeout-method thread > $O/rest.log 2>&1; rc=$?
tail -3 $O/rest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/rest.log | head -20; exit $rc; }
