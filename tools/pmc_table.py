#!/usr/bin/env python3
"""Per-launch averages of every PMC counter in rocprofv3 counter_collection CSVs, per kernel.

  python tools/pmc_table.py gpurun_out/prof/r02d_deep* [--kernel hg_trace_stream_kernel]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="hg_trace_stream_kernel<false")
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    dispatches = collections.defaultdict(set)
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if a.kernel not in r["Kernel_Name"]:
                    continue
                name = r["Counter_Name"]
                tot[name] += float(r["Counter_Value"])
                dispatches[name].add((f, r["Dispatch_Id"]))
    for name in sorted(tot):
        n = len(dispatches[name])
        print(f"{name:40s} {tot[name] / n:16.6g}   ({n} launches)")


if __name__ == "__main__":
    main()
