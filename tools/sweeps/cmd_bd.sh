set -u
export TMPDIR=/tmp
SWEEP_TIMEOUT=200 bash tools/sweep.sh tools/sweeps/sweep_r02_bd.txt || exit $?
mkdir -p gpurun_out/prof
for v in fc pm; do
HALOGEN_LIB=$PWD/variants/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bc_$v -o s --output-format csv -- python3 bench.py --steps 8 --no-framed --no-cpu-baseline > gpurun_out/prof/bc_$v.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bc_base -o s --output-format csv -- python3 bench.py --steps 8 --no-framed --no-cpu-baseline > gpurun_out/prof/bc_base.log 2>&1 || exit $?
