# PMC of the queue form against the per-tile waves on C3 at N=1 (HG_OPT_QUEUE_FILL 0 vs 64), then the teardown factors
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/qpmc
mkdir -p $O
for f in 0 64; do
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
             "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_LDS"; do
    n=$(echo $grp | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/f${f}_$n -o p --output-format csv -- python3 bench.py --queue-fill $f \
        --steps 2 --warmup 1 --no-per-frame --no-cpu-baseline --no-framed --no-fast-bvh --no-counters > $O/f${f}_$n.log 2>&1 || { tail -5 $O/f${f}_$n.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for f in (0, 64):
    tot = collections.Counter(); n = collections.Counter()
    for path in glob.glob(f"gpurun_out/qpmc/f{f}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if "trace_stream_kernel" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"fill {f}:", {k: f"{v:.4g}" for k, v in sorted(tot.items())})
PY
CASES="r05pre_trace HG_TD_DEFER_EVENTS=1;r05pre_trace HG_TD_DEFER_BUFS=1" bash tools/gpu_teardown_r05pre.sh
