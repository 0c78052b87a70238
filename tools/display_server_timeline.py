#!/usr/bin/env python3
"""The per-frame display chain of the render server (bench.py --per-frame-only --display sync|pipelined under rocprofv3
--kernel-trace --memory-copy-trace): for the last N frames, the gate (its wait for the frame's count), the blend, the
untile / pack and the device-to-host copy of the display image, the gaps between them, and the period between
consecutive frames' copies (the host's display loop).  With the server tracing ahead (HG_OPT_SERVER_AHEAD) a frame's
count is usually there when its gate starts, so the chain is what is left of a frame's display latency.

Usage: display_server_timeline.py DIR [N_LAST]   (DIR holds the *kernel_trace.csv and *memory_copy_trace.csv)"""
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 64
K = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
           for r in csv.DictReader(open(next(d.rglob("*kernel_trace.csv")))))
copies = []
mc = list(d.rglob("*memory_copy_trace.csv"))
if mc:
    copies = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(mc[0]))
                    if "DEVICE_TO_HOST" in r["Direction"])
ms = 1e6


def mean(v):
    return sum(v) / len(v) if v else float("nan")


gate = [k for k in K if "server_gate" in k[2]][-n_last:]
blend = [k for k in K if "server_blend" in k[2]][-n_last:]
untile = [k for k in K if "untile" in k[2]]
print(f"frames {len(gate)} (gates), blends {len(blend)}, untiles {len(untile)}, D2H copies {len(copies)}")
if not gate:
    sys.exit(0)
t0 = gate[0][0]
untile = [u for u in untile if u[0] >= t0]
copies = [c for c in copies if c[0] >= t0]
print(f"gate span (waiting for the frame's count) mean {mean([(g[1] - g[0]) / ms for g in gate]):.4f} ms, "
      f"max {max((g[1] - g[0]) / ms for g in gate):.4f}")
print(f"gate end -> blend start {mean([(b[0] - g[1]) / ms for g, b in zip(gate, blend)]):.4f} ms; "
      f"blend span {mean([(b[1] - b[0]) / ms for b in blend]):.4f} ms")


def first_after(seq, t):
    for x in seq:
        if x[0] >= t:
            return x
    return None


bu, uc, cspan, cu = [], [], [], []
for b in blend:
    u = first_after(untile, b[1])
    if not u:
        continue
    bu.append((u[0] - b[1]) / ms)
    cu.append((u[1] - u[0]) / ms)
    c = first_after(copies, u[1])
    if c:
        uc.append((c[0] - u[1]) / ms)
        cspan.append((c[1] - c[0]) / ms)
print(f"blend end -> untile start {mean(bu):.4f} ms; untile span {mean(cu):.4f} ms")
print(f"untile end -> copy start {mean(uc):.4f} ms; copy span {mean(cspan):.4f} ms")
if len(copies) > 1:
    per = [(b[1] - a[1]) / ms for a, b in zip(copies, copies[1:])]
    print(f"copy end -> next copy end (display period) mean {mean(per):.4f} ms")
    nxt = []
    for c in copies:
        g = first_after(gate, c[1])
        if g:
            nxt.append((g[0] - c[1]) / ms)
    print(f"copy end -> next gate start (host: end of readback, next render call) {mean(nxt):.4f} ms")
