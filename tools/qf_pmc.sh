set -u
export BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-framed --no-per-frame"
TAG=qfbase bash tools/pmc_deep.sh || exit $?
HALOGEN_LIB=variants/lib_qf1.so TAG=qf1 bash tools/pmc_deep.sh || exit $?
python3 tools/pmc_table.py gpurun_out/prof/deep*_qfbase > gpurun_out/qf_pmc_base.txt 2>&1
python3 tools/pmc_table.py gpurun_out/prof/deep*_qf1 > gpurun_out/qf_pmc_qf1.txt 2>&1
