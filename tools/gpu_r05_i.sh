#!/bin/bash
# PMC passes of the render server at the strict per-frame point (per dispatch = per server lifetime), to set beside
# the batched kernel's (profiles/r05p_td_attribution.json)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof/attrib_r05s
mkdir -p "$OUT"
k=0
while read -r counters; do
  [ -z "$counters" ] && continue
  k=$((k + 1))
  timeout -s KILL 90 rocprofv3 --pmc $counters -d "$OUT/SV_p${k}" -o pmc --output-format csv -- \
      python3 bench.py --per-frame-only --steps 2 --server 2 > "$OUT/SV_p${k}.log" 2>&1
  rc=$?; echo "pass $k rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/SV_p${k}.log"; exit $rc; }
done <<'LIST'
TD_TD_BUSY_sum TD_TC_STALL_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum GRBM_GUI_ACTIVE
TD_LOAD_WAVEFRONT_sum TD_COALESCABLE_WAVEFRONT_sum TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum
TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_LATENCY_sum
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU
LIST
