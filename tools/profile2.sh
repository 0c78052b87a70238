#!/bin/bash
# rocprofv3 kernel stats + two PMC groups for one bench configuration.  Usage: TAG=x ARGS="..." profile2.sh
set -u
TAG=${TAG:-x}
ARGS=${ARGS:---steps 1 --warmup 1 --frames-per-step 16 --no-cpu-baseline}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 420 rocprofv3 "$@" -d "$OUT/${TAG}_${name}" -o "$name" --output-format csv -- python3 bench.py $ARGS \
      > "$OUT/${TAG}_${name}.log" 2>&1
  local rc=$?; echo "$TAG $name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/${TAG}_${name}.log"; exit $rc; }
}
run stats --kernel-trace --stats
run valu --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run mem --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY TCC_HIT_sum TCC_MISS_sum
cat "$OUT/${TAG}_stats/stats_kernel_stats.csv"
