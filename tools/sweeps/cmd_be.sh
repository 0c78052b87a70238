set -u
export TMPDIR=/tmp
HALOGEN_LIB=$PWD/variants/lib_pm2.so timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_pm2.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pm2.log; [ $rc -eq 0 ] || exit $rc
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r02_be.txt || exit $?
bash tools/pmc_write_ab.sh fc2 pm2 || exit $?
mkdir -p gpurun_out/prof
HALOGEN_LIB=$PWD/variants/lib_pm2.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/be_pm2 -o s --output-format csv -- python3 bench.py --steps 8 --no-framed --no-cpu-baseline > gpurun_out/prof/be_pm2.log 2>&1 || exit $?
