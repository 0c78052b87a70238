#!/bin/bash
# rocprofv3 passes for each config in $CONFIGS (kernel trace + stats; then one pass per PMC group), the timed
# (counter-free) kernels of bench.py's main measurement only.  Each step has its own time limit; any failure ends the
# script.  Output: gpurun_out/prof/<TAG>_<cfg>_<pass>/.
set -u
TAG=${TAG:-r04}
CONFIGS=${CONFIGS:-C3 C3F C2 C5}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in $CONFIGS; do
  ARGS="--config $cfg --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --no-framed --no-per-frame --no-counters ${BENCH_EXTRA:-}"
  run() {  # name, extra rocprofv3 args...
    local name=$1; shift
    timeout -k 10 240 rocprofv3 "$@" -d "$OUT/${TAG}_${cfg}_${name}" -o "$name" --output-format csv -- \
        python3 bench.py $ARGS > "$OUT/${TAG}_${cfg}_${name}.log" 2>&1
    local rc=$?; echo "$cfg $name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/${TAG}_${cfg}_${name}.log"; exit $rc; }
  }
  run stats --kernel-trace --stats
  run fetch --pmc FETCH_SIZE
  run write --pmc WRITE_SIZE
  run valu --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
  run mem --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY TCC_HIT_sum TCC_MISS_sum
  run td --pmc TA_BUSY_avr TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
  grep -h '"value"' "$OUT/${TAG}_${cfg}_stats.log" | tail -1 | cut -c1-200
done
