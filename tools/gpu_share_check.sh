set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/share
timeout -k 10 600 python -u -m pytest tests/test_gpu_per_frame.py tests/test_gpu_comm.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/share/tests.log 2>&1 || { tail -30 gpurun_out/share/tests.log; exit 1; }
tail -2 gpurun_out/share/tests.log
POINTS="8:-1:-1 4:-1:-1 2:-1:-1" STEPS=8 bash tools/gpu_strong_coalesce.sh
