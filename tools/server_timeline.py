#!/usr/bin/env python3
"""Per-frame timeline of the render server (bench.py --per-frame-only --server 1 under rocprofv3 --kernel-trace): the
server launches (one per lifetime), and for the last N frames the gate (start -> end: how long the frame's count took
to arrive after the gate began polling), the blend and, with a display, the untile kernel, with the gaps between them.

Usage: server_timeline.py DIR [N_LAST]   (DIR holds pf_kernel_trace.csv)"""
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 64
K = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
           for r in csv.DictReader(open(next(d.rglob("*kernel_trace.csv")))))
ms = 1e6


def mean(v):
    return sum(v) / len(v) if v else float("nan")


server = [k for k in K if "trace_stream_kernel" in k[2] and "true>" in k[2].split(",")[-1]]
gate = [k for k in K if "server_gate" in k[2]][-n_last:]
blend = [k for k in K if "server_blend" in k[2]][-n_last:]
untile = [k for k in K if "untile" in k[2]]
print(f"server launches {len(server)}: spans (ms) {[round((k[1] - k[0]) / ms, 2) for k in server][:8]}")
print(f"gates {len(gate)}: mean span {mean([(g[1] - g[0]) / ms for g in gate]):.4f} ms")
print(f"blends {len(blend)}: mean span {mean([(b[1] - b[0]) / ms for b in blend]):.4f} ms, "
      f"gate end -> blend start {mean([(b[0] - g[1]) / ms for g, b in zip(gate, blend)]):.4f} ms")
if len(gate) > 1:
    print(f"frame period (gate end to gate end) {mean([(b[1] - a[1]) / ms for a, b in zip(gate, gate[1:])]):.4f} ms")
if untile:
    ut = [u for u in untile if u[0] >= gate[0][0]]
    print(f"untiles {len(ut)}: mean span {mean([(u[1] - u[0]) / ms for u in ut]):.4f} ms")
    nxt = []
    for b in blend:
        after = [u for u in ut if u[0] >= b[1]]
        if after:
            nxt.append((after[0][0] - b[1]) / ms)
    print(f"blend end -> next untile start {mean(nxt):.4f} ms")
others = {}
for k in K:
    if k[0] < (gate[0][0] if gate else 0):
        continue
    name = k[2].split("(")[0][:60]
    others.setdefault(name, []).append((k[1] - k[0]) / ms)
for name, v in sorted(others.items(), key=lambda x: -sum(x[1])):
    print(f"  {name:60s} n={len(v):5d} mean {mean(v):.4f} ms total {sum(v):.2f} ms")
