set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wave_units.py tests/test_gpu_per_frame.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06a_pytest.log 2>&1 || { tail -30 gpurun_out/r06a_pytest.log; exit 1; }
tail -2 gpurun_out/r06a_pytest.log
bash tools/gpu_emulate.sh && bash tools/gpu_launch.sh
