#!/bin/bash
# L1 traffic of the timed C3 trace kernel, default library vs variants/lib_aos.so (one --pmc pass each), then C2 pairs.
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 2 --no-cpu-baseline --no-framed --no-per-frame --no-counters"
for v in default aos; do
  if [ $v = default ]; then unset HALOGEN_LIB; else export HALOGEN_LIB=variants/lib_aos.so; fi
  timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE \
      -d gpurun_out/prof/aos_$v -o l1 --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/aos_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
unset HALOGEN_LIB
A="--config C2 --steps 8 --warmup 3 --no-framed --no-per-frame --no-counters"
printf '%s\n' "$A" "HALOGEN_LIB=variants/lib_aos.so $A" "$A" "HALOGEN_LIB=variants/lib_aos.so $A" > gpurun_out/aos_c2.txt
bash tools/sweep.sh gpurun_out/aos_c2.txt 2>&1 | tail -4
