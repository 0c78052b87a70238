#!/usr/bin/env python3
"""Per-frame instruction mix of the streaming kernel's forms (tools/pmc_instmix.sh output): sums every dispatch of the
counter-free streaming kernel in each run and divides by the frames it traced (batched: 64 per launch; the queue and the
server: the frames the run rendered, from its bench log's frame count, warm-up included).

  python3 tools/instmix.py gpurun_out/prof/instmix_<TAG>"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
W, H = 1920, 1080
rows = {}
for form in ("batched", "queue", "server"):
    f = glob.glob(os.path.join(d, form, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    tot, disp = collections.defaultdict(float), set()
    for r in csv.DictReader(open(f[0])):
        if not r["Kernel_Name"].startswith("void hg_trace_stream_kernel<false"):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
    if form == "batched":
        frames = 64 * len(disp)
    else:  # warm-up step + timed step of --frames-per-step 1-frame calls
        frames = 2 * 64
    rows[form] = {"dispatches": len(disp), "frames": frames,
                  **{k: v / frames for k, v in sorted(tot.items())}}
keys = sorted({k for r in rows.values() for k in r if k.startswith("SQ_")})
print(f"{'per frame':24s}" + "".join(f"{f:>14s}" for f in rows))
for k in ["dispatches", "frames"] + keys:
    print(f"{k:24s}" + "".join(f"{rows[f].get(k, 0):14.4g}" for f in rows))
if "--json" in sys.argv:
    json.dump(rows, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
