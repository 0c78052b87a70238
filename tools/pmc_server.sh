#!/bin/bash
# PMC passes of the render server's trace kernel ("the server cannot be PMC-profiled"): C3's
# strict per-frame loop with the server forced (bench.py --per-frame-only --server 2).  Under --pmc the profiler
# serialises kernels, so a frame's gate cannot run beside the server: each lifetime traces what was posted (the host
# blocks on the ring after 16 frames), closes itself after HG_OPT_SERVER_IDLE_US of nothing posted (the close
# handshake), then its gates pass at once and the next post starts a new lifetime.  Same counter groups as
# tools/pmc_attrib.sh; each pass under its own limit, any failure ends the script.  HALOGEN_SERVER_SERIAL=1 makes
# every gate wait for its lifetime's end (the profiler would otherwise run a gate before the server it waits for).
#   TAG=r06s bash tools/pmc_server.sh ; python3 tools/pmc_attrib.py gpurun_out/prof/server_r06s --kernel <server symbol>
set -u
TAG=${TAG:-server}
OUT=$PWD/gpurun_out/prof/server_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
k=0
while read -r counters; do
  [ -z "$counters" ] && continue
  k=$((k + 1))
  HALOGEN_SERVER_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc $counters -d "$OUT/C3S_p${k}" -o pmc --output-format csv -- \
      python3 bench.py --config C3 --per-frame-only --server 2 --server-idle-us 2000 --server-ahead 0 --launch-frames 1 \
      --frames-per-step 64 --steps 1 \
      --no-counters --no-cpu-baseline > "$OUT/C3S_p${k}.log" 2>&1
  rc=$?; echo "pass $k rc=$rc ($counters)"; [ $rc -eq 0 ] || { tail -5 "$OUT/C3S_p${k}.log"; exit $rc; }
done <<'LIST'
TD_TD_BUSY_sum TD_TC_STALL_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum GRBM_GUI_ACTIVE
TD_LOAD_WAVEFRONT_sum TD_COALESCABLE_WAVEFRONT_sum TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum
TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_LATENCY_sum
TCP_TOTAL_READ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU
LIST
