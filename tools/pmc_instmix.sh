#!/bin/bash
# Instruction mix per launch of the streaming kernel's forms (one rocprofv3 --pmc pass each, under its own limit):
#   batched  C3, hg_render(64) per step (per-tile waves)
#   queue    C3, 1-frame launches (the persistent queue form; --server 0, coalesce 1)
#   server   C3, 1-frame calls through the render server (--server 2; HALOGEN_SERVER_SERIAL=1, idle close 2 ms, no frames
#            traced ahead: a stop abandons none)
# Wave-level VMEM reads / writes, LDS, SMEM, VALU and waves: per frame they say what each form adds to the batched one.
set -u
OUT=$PWD/gpurun_out/prof/instmix_${TAG:-x}
mkdir -p "$OUT"
export TMPDIR=/tmp
C="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU SQ_WAVES SQ_INSTS_FLAT SQ_INSTS_SALU"
B="python3 bench.py --config C3 --no-cpu-baseline --no-framed --no-fast-bvh --no-counters"
run() {
  local tag=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc $C -d "$OUT/$tag" -o pmc --output-format csv -- "$@" > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$tag.log"; exit $rc; }
}
run batched $B --steps 2 --warmup 1 --no-per-frame
run queue $B --per-frame-only --server 0 --launch-frames 1 --frames-per-step 64 --steps 1
HALOGEN_SERVER_SERIAL=1 run server $B --per-frame-only --server 2 --server-idle-us 2000 --server-ahead 0 --launch-frames 1 \
    --frames-per-step 64 --steps 1
