#!/usr/bin/env python3
"""profiles/<TAG>_perframe_summary.json from tools/profile_perframe.sh's rocprofv3 runs (bench.py --per-frame-only at
coalesce 1 and 32): per kernel calls, average duration and the mean period between launch starts, plus the bench line.
    python3 tools/summarize_perframe.py r03e"""
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def kname(raw: str) -> str:
    return raw.split("(")[0].replace("void ", "").strip()


def main():
    tag = sys.argv[1]
    src = ROOT / "gpurun_out" / "prof"
    out = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --per-frame-only --steps 2 --coalesce {1,32} "
                      "[--server 0] (C3, 2 x 64 hg_render(1) calls after one 64-frame warm-up)"}
    runs = [co for co in ("1", "1_srv0", "32") if (src / f"{tag}_perframe_co{co}").exists()]
    for co in runs:
        d = src / f"{tag}_perframe_co{co}"
        stats = next(d.glob("*_kernel_stats.csv"))
        shutil.copy(stats, ROOT / "profiles" / f"{tag}_perframe_co{co}_kernel_stats.csv")
        starts = {}
        for r in csv.DictReader(open(next(d.glob("*_kernel_trace.csv")))):
            starts.setdefault(kname(r["Kernel_Name"]), []).append(int(r["Start_Timestamp"]))
        kernels = {}
        for r in csv.DictReader(open(stats)):
            k = kname(r["Name"])
            e = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
            s = sorted(starts.get(k, []))
            if len(s) > 1:
                e["start_period_ms"] = (s[-1] - s[0]) / (len(s) - 1) / 1e6
            kernels[k] = e
        bench = [json.loads(x) for x in open(src / f"{tag}_perframe_co{co}.log") if x.startswith('{"per_frame_only"')]
        out[f"coalesce_{co}"] = {"bench": bench[-1] if bench else None, "kernels": kernels}
    (ROOT / "profiles" / f"{tag}_perframe_summary.json").write_text(json.dumps(out, indent=1) + "\n")
    for co in runs:
        print(co, out[f"coalesce_{co}"]["bench"])


if __name__ == "__main__":
    main()
