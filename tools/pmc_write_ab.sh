#!/bin/bash
# WRITE_SIZE of the timed stream kernel, default library vs variants/lib_<name>.so (one --pmc pass each).
#   bash tools/pmc_write_ab.sh name...
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcw
for v in default "$@"; do
  if [ $v = default ]; then unset HALOGEN_LIB; else export HALOGEN_LIB=variants/lib_$v.so; fi
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw/$v -o w --output-format csv -- python3 bench.py \
      --steps 4 --warmup 1 --no-cpu-baseline --no-framed --no-per-frame --no-counters > gpurun_out/pmcw/$v.log 2>&1 || exit 1
  echo "$v ok"
done
