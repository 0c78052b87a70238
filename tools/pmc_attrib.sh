#!/bin/bash
# Where the texture-data (TD) unit's cycles per vector-memory instruction go: the timed trace
# kernel of each config in CONFIGS, one rocprofv3 --pmc pass per counter group (within gfx950's per-block limits:
# 8 SQ, 4 TCP, 2 TA, 2 TD, 2 GRBM), each under its own time limit; any failure ends the script.
#   TAG=r05p CONFIGS="C3 C3F" bash tools/pmc_attrib.sh ; python3 tools/pmc_attrib.py gpurun_out/prof/attrib_r05p
set -u
TAG=${TAG:-attrib}
CONFIGS=${CONFIGS:-C3 C3F}
OUT=$PWD/gpurun_out/prof/attrib_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in $CONFIGS; do
  k=0
  while read -r counters; do
    [ -z "$counters" ] && continue
    k=$((k + 1))
    timeout -s KILL 90 rocprofv3 --pmc $counters -d "$OUT/${cfg}_p${k}" -o pmc --output-format csv -- \
        python3 bench.py --config "$cfg" --steps 2 --warmup 1 --no-cpu-baseline --no-framed --no-per-frame \
        --no-counters --no-fast-bvh > "$OUT/${cfg}_p${k}.log" 2>&1
    rc=$?; echo "$cfg pass $k rc=$rc ($counters)"; [ $rc -eq 0 ] || { tail -5 "$OUT/${cfg}_p${k}.log"; exit $rc; }
  done <<'LIST'
TD_TD_BUSY_sum TD_TC_STALL_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum GRBM_GUI_ACTIVE
TD_LOAD_WAVEFRONT_sum TD_COALESCABLE_WAVEFRONT_sum TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum
TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_LATENCY_sum
TCP_TOTAL_READ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU
LIST
done
