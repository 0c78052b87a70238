#!/bin/bash
# rocprofv3 passes over a short bench run (kernel trace + stats; then one pass per PMC group).  Each step has
# its own time limit; any failure ends the script.  Output: gpurun_out/prof/<tag>_*.
set -u
TAG=${TAG:-r01}
ARGS=${BENCH_ARGS:---steps 16 --warmup 2 --no-cpu-baseline --no-framed}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, extra rocprofv3 args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -d "$OUT/${TAG}_${name}" -o "$name" --output-format csv -- python3 bench.py $ARGS \
      > "$OUT/${TAG}_${name}.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/${TAG}_${name}.log"; exit $rc; }
}
run stats --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run valu --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run mem --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY TCC_HIT_sum TCC_MISS_sum
run td --pmc TA_BUSY_avr TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
find "$OUT" -name "*.csv" | head -50
