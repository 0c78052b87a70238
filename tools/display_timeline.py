#!/usr/bin/env python3
"""Per-frame timeline of a per-frame display run (bench.py --per-frame-only --display pipelined under rocprofv3
--kernel-trace --memory-copy-trace): for the last N frames, each frame's trace launch, blend, untile and D2H copy in
order, and the stage-to-stage delays averaged over the frames:

  trace span            the frame's trace kernel, start to end
  trace end -> blend    the in-order blend on the context stream
  blend end -> untile   the display untile kernel
  untile end -> copy    the D2H copy's start, and its duration
  copy end -> next+d    the next trace launch d frames later (host: readback_end of this frame, then render)

Usage: display_timeline.py DIR [N_LAST]   (DIR holds pf_kernel_trace.csv and pf_memory_copy_trace.csv)"""
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 64
kr = list(csv.DictReader(open(d / "pf_kernel_trace.csv")))
cr = list(csv.DictReader(open(d / "pf_memory_copy_trace.csv"))) if (d / "pf_memory_copy_trace.csv").exists() else []
K = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Queue_Id"])) for r in kr)
C = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"]) for r in cr
           if "DEVICE_TO_HOST" in r["Direction"])
trace = [k for k in K if "trace_stream_kernel" in k[2] or "trace_regen_kernel" in k[2]]
blend = [k for k in K if "blend_frames" in k[2]]
untile = [k for k in K if "untile" in k[2]]
trace, blend = trace[-n_last:], blend[-n_last:]
untile = untile[-n_last:]
C = C[-n_last:]
ms = 1e6


def mean(v):
    return sum(v) / len(v) if v else float("nan")


n = min(len(trace), len(blend))
print(f"frames {n}: traces {len(trace)} blends {len(blend)} untiles {len(untile)} D2H copies {len(C)}")
t0, t1 = trace[0][0], max(b[1] for b in blend)
print(f"window {(t1 - t0) / ms:.3f} ms, {(t1 - t0) / ms / n:.4f} ms per frame")
spans = [(t[1] - t[0]) / ms for t in trace]
print(f"trace span mean {mean(spans):.3f} ms  min {min(spans):.3f}  max {max(spans):.3f}")
print(f"trace start-to-start mean {mean([(b[0] - a[0]) / ms for a, b in zip(trace, trace[1:])]):.4f} ms")
print(f"trace end -> blend start   {mean([(b[0] - t[1]) / ms for t, b in zip(trace, blend)]):.4f} ms;"
      f" blend span {mean([(b[1] - b[0]) / ms for b in blend]):.4f} ms")
if len(untile) >= n and len(C) >= n:
    print(f"blend end -> untile start  {mean([(u[0] - b[1]) / ms for b, u in zip(blend, untile)]):.4f} ms;"
          f" untile span {mean([(u[1] - u[0]) / ms for u in untile]):.4f} ms")
    print(f"untile end -> copy start   {mean([(c[0] - u[1]) / ms for u, c in zip(untile, C)]):.4f} ms;"
          f" copy span {mean([(c[1] - c[0]) / ms for c in C]):.4f} ms")
    for dd in (1, 2, 7, 8):
        if n > dd:
            print(f"copy end (k) -> trace start (k+{dd}) {mean([(trace[i + dd][0] - C[i][1]) / ms for i in range(n - dd)]):.4f} ms")
    print(f"trace start -> copy end (latency) {mean([(c[1] - t[0]) / ms for t, c in zip(trace, C)]):.3f} ms")
# concurrency of traces
pts = sorted([(t[0], 1) for t in trace] + [(t[1], -1) for t in trace])
cur, last, hist = 0, pts[0][0], {}
for t, dlt in pts:
    hist[cur] = hist.get(cur, 0) + t - last
    cur += dlt
    last = t
tot = sum(hist.values())
print("traces in flight (time share):", " ".join(f"{k}:{v / tot:.2f}" for k, v in sorted(hist.items())))
grids = sorted(set(int(r["Grid_Size_X"]) // 64 for r in kr if "trace_stream" in r["Kernel_Name"]))
print("waves per trace launch:", grids[:12])
