#!/bin/bash
# Memory-pipeline counters of the timed trace kernel (TA/TD/TCP/SQ levels), one rocprofv3 --pmc pass per group,
# each under its own time limit; any failure ends the script.  Output: gpurun_out/prof/deep<k>_<TAG>/ (outside the summarizer's <TAG>_* glob).
#   TAG=r02d bash tools/pmc_deep.sh ; python tools/pmc_table.py gpurun_out/prof/deep*_r02d
set -u
TAG=${TAG:-deep}
ARGS=${BENCH_ARGS:---steps 4 --warmup 1 --no-cpu-baseline --no-framed}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
k=0
while read -r counters; do
  [ -z "$counters" ] && continue
  k=$((k + 1))
  timeout -s KILL 120 rocprofv3 --pmc $counters -d "$OUT/deep${k}_${TAG}" -o deep --output-format csv -- \
      python3 bench.py $ARGS > "$OUT/deep${k}_${TAG}.log" 2>&1
  rc=$?; echo "pass $k rc=$rc ($counters)"; [ $rc -eq 0 ] || { tail -5 "$OUT/deep${k}_${TAG}.log"; exit $rc; }
done <<'LIST'
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum
TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES
SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES
LIST
