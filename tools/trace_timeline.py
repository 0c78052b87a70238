"""Timeline of a rocprofv3 kernel trace (pf_kernel_trace.csv): per kernel name the launches, their mean span, and for
the trace kernel the concurrency (launches in flight) over the timed part, the gaps between consecutive launch starts
and what runs between a launch's end and the next start on the same queue.  Usage: trace_timeline.py TRACE.csv [N_LAST]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Queue_Id"]), int(r["Grid_Size_X"]))
      for r in rows]
ev.sort()
trace = [e for e in ev if "trace_stream_kernel" in e[2] or "trace_regen_kernel" in e[2]]
if n_last:
    trace = trace[-n_last:]
t0, t1 = trace[0][0], max(e[1] for e in trace)
print(f"trace launches {len(trace)}, window {(t1 - t0) / 1e6:.3f} ms, per launch {(t1 - t0) / 1e6 / len(trace):.4f} ms")
spans = [(e[1] - e[0]) / 1e6 for e in trace]
print(f"span mean {sum(spans) / len(spans):.3f} ms min {min(spans):.3f} max {max(spans):.3f}")
starts = [e[0] for e in trace]
gaps = [(b - a) / 1e6 for a, b in zip(starts, starts[1:])]
print(f"start-to-start mean {sum(gaps) / len(gaps):.4f} ms")
# concurrency histogram (time-weighted)
pts = sorted([(e[0], 1) for e in trace] + [(e[1], -1) for e in trace])
cur, last, hist = 0, pts[0][0], defaultdict(float)
for t, d in pts:
    hist[cur] += t - last
    cur += d
    last = t
tot = sum(hist.values())
print("in flight (time share):", " ".join(f"{k}:{v / tot:.3f}" for k, v in sorted(hist.items())))
others = defaultdict(list)
for e in ev:
    if e[0] >= t0 and e[1] <= t1 and e not in trace:
        others[e[2][:40]].append((e[1] - e[0]) / 1e6)
for k, v in others.items():
    print(f"  {k}: {len(v)} launches, mean {sum(v) / len(v):.4f} ms, max {max(v):.4f} ms")
grid = defaultdict(int)
for e in trace:
    grid[e[4] // 64] += 1
print("waves per trace launch:", dict(sorted(grid.items())))
