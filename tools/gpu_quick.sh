set -u
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
SWEEP_TIMEOUT=300 bash tools/sweep.sh tools/sweeps/sweep40.txt || exit $?
bash tools/util.sh
