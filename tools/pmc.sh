#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass) over one bench configuration; prints per-kernel sums.
# Usage: TAG=x ARGS="bench args" bash tools/pmc.sh "GROUP1" "GROUP2" ...   (a GROUP is a space-separated list)
set -u
TAG=${TAG:-x}
ARGS=${ARGS:---steps 1 --warmup 1 --frames-per-step 16 --no-cpu-baseline}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $grp -d "$OUT/${TAG}_pmc$i" -o pmc --output-format csv -- python3 bench.py $ARGS \
      > "$OUT/${TAG}_pmc$i.log" 2>&1
  rc=$?; echo "$TAG pass $i rc=$rc ($grp)"; [ $rc -eq 0 ] || { tail -20 "$OUT/${TAG}_pmc$i.log"; exit $rc; }
done
python3 - "$OUT" "$TAG" <<'PY'
import csv, collections, glob, sys
out, tag = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(f"{out}/{tag}_pmc*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if "rocclr" in k:
        continue
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:40s} {x:.4g}")
PY
