#!/usr/bin/env python3
"""Summarise one rocprofv3 profiling session of bench.py (tools/profile.sh TAG=...) into profiles/.

  python tools/summarize_profile.py TAG [--frames-per-launch 64] [--config C3 --width 1920 --height 1080]

Writes profiles/<TAG>_kernel_stats.csv (the --stats table as produced), profiles/<TAG>_summary.json (per-kernel
average duration and PMC counters per launch) and, for the production kernel, profiles/pmc_traffic.json, read
by bench.py as roofline.traffic.

HBM traffic per launch follows /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane loads (our node / triangle
loads are global_load_dwordx4, 16 B per lane), so fetch bytes = FETCH_SIZE x 1024 x 2; WRITE_SIZE is exact for
16-B-per-lane stores (the accumulator float4 stores).  The counters sit on the L2's fabric side, so Infinity
Cache hits are included: the figure is an upper bound of DRAM traffic.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import shutil
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
N_CU, N_XCD = 256, 8  # MI355X


def kname(raw: str) -> str:
    return raw.replace("void ", "").split("(")[0]


def interval_union(spans) -> float:
    """Total length covered by the (start, end) intervals (the time at least one of them runs)."""
    busy, lo, hi = 0, None, None
    for x0, x1 in sorted(spans):
        if hi is None or x0 > hi:
            if hi is not None:
                busy += hi - lo
            lo, hi = x0, x1
        else:
            hi = max(hi, x1)
    if hi is not None:
        busy += hi - lo
    return busy


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--src", default=str(ROOT / "gpurun_out" / "prof"))
    ap.add_argument("--frames-per-launch", type=int, default=64)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--command", default="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline")
    ap.add_argument("--library-sha256", default="", help="sha256 of the libhalogen_hip.so the profile ran")
    ap.add_argument("--warmup-launches", type=int, default=2,
                    help="launches of the production kernel before bench.py's timed region (its --warmup)")
    ap.add_argument("--traffic-out", default="pmc_traffic.json",
                    help="file under profiles/ for the production kernel's per-launch counters (bench.py reads "
                         "pmc_traffic.json for the headline config, pmc_traffic_<config>.json for the others)")
    a = ap.parse_args()
    src = Path(a.src)
    out = ROOT / "profiles"
    out.mkdir(exist_ok=True)

    stats_csv = src / f"{a.tag}_stats" / "stats_kernel_stats.csv"
    shutil.copy(stats_csv, out / f"{a.tag}_kernel_stats.csv")
    stats = {}
    for r in csv.DictReader(open(stats_csv)):
        stats[kname(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                   "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6}

    # per-launch durations from the kernel trace: the bench's first launch (warmup) runs in tile-index order, the
    # later ones in the cost order it recorded (HG_OPT_TILE_ORDER), so the timed launches are the ones after it
    trace_csv = src / f"{a.tag}_stats" / "stats_kernel_trace.csv"
    if trace_csv.exists():
        durs = collections.defaultdict(list)
        spans = collections.defaultdict(list)
        for r in csv.DictReader(open(trace_csv)):
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            durs[kname(r["Kernel_Name"])].append((t1 - t0) / 1e6)
            spans[kname(r["Kernel_Name"])].append((t0, t1))
        for k, v in durs.items():
            if k in stats:
                stats[k]["launch_ms"] = v
                if len(v) > 1:
                    stats[k]["avg_ms_after_first"] = sum(v[1:]) / (len(v) - 1)
                if len(v) > a.warmup_launches:
                    # the launches of bench.py's timed region: what its HIP events average (roofline.mean_launch_ms)
                    t = v[a.warmup_launches:]
                    stats[k]["avg_ms_timed"] = sum(t) / len(t)
                    # launches on the two trace streams overlap: the union of their intervals per launch is the
                    # kernel's device time per launch (bench.py: trace_busy_ms / trace_launches)
                    iv = spans[k][a.warmup_launches:]
                    stats[k]["avg_ms_timed_union"] = interval_union(iv) / 1e6 / len(iv)
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in sorted(glob.glob(str(src / f"{a.tag}_*" / "*_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k][r["Counter_Name"]].add(r["Dispatch_Id"])
    kernels = {}
    for k in sorted(set(stats) | set(sums)):
        pmc = {c: v / max(len(calls[k][c]), 1) for c, v in sums[k].items()}
        d = {"stats": stats.get(k), "pmc_per_launch": pmc}
        if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
            fetch = pmc["FETCH_SIZE"] * 1024 * 2
            write = pmc["WRITE_SIZE"] * 1024
            d["hbm_bytes_per_launch"] = fetch + write
            d["fetch_bytes_per_launch"] = fetch
            d["write_bytes_per_launch"] = write
        if "TCC_HIT_sum" in pmc and "TCC_MISS_sum" in pmc:
            d["l2_hit_rate"] = pmc["TCC_HIT_sum"] / max(pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"], 1)
        if "SQ_WAVE_CYCLES" in pmc and pmc["SQ_WAVE_CYCLES"] > 0:
            wc = pmc["SQ_WAVE_CYCLES"]
            d["wave_cycle_split"] = {"wait_any": pmc.get("SQ_WAIT_ANY", 0) / wc,
                                     "wait_inst_any": pmc.get("SQ_WAIT_INST_ANY", 0) / wc}
        if "TD_TD_BUSY_sum" in pmc and pmc.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE sums the 8 XCDs' cycles; the TD/TA counters sum (or average) over the 256 CUs (MI355X)
            cyc = pmc["GRBM_GUI_ACTIVE"] / N_XCD
            d["vmem_unit_busy"] = {"td_busy": pmc["TD_TD_BUSY_sum"] / (N_CU * cyc),
                                   "td_stalled_on_l1": pmc.get("TD_TC_STALL_sum", 0) / (N_CU * cyc),
                                   "ta_busy": pmc.get("TA_BUSY_avr", 0) / cyc}
        kernels[k] = d
    summary = {"tag": a.tag, "command": f"rocprofv3 --kernel-trace --stats | --pmc <group> -- {a.command}",
               "config": a.config, "width": a.width, "height": a.height,
               "frames_per_launch": a.frames_per_launch, "kernels": kernels}
    (out / f"{a.tag}_summary.json").write_text(json.dumps(summary, indent=1) + "\n")
    # the production kernel: the counter-free trace kernel that ran longest (the bench's timed launches)
    # (template arguments: <kCounters> or <kCounters, variant>; production = kCounters false)
    prods = [k for k in kernels if k.startswith("hg_trace") and "<false" in k and kernels[k]["stats"]]
    PROD = max(prods, key=lambda k: kernels[k]["stats"]["calls"] * kernels[k]["stats"]["avg_ms"]) if prods else ""
    if PROD in kernels and "hbm_bytes_per_launch" in kernels[PROD]:
        k = kernels[PROD]
        pmc = k["pmc_per_launch"]
        t = {"tag": a.tag, "summary": f"profiles/{a.tag}_summary.json", "kernel": PROD, "config": a.config,
             "width": a.width, "height": a.height, "frames_per_launch": a.frames_per_launch,
             "library_sha256": a.library_sha256,
             "hbm_bytes_per_launch": k["hbm_bytes_per_launch"],
             "write_bytes_per_launch": k.get("write_bytes_per_launch"),
             "note": "FETCH_SIZE*1024*2 + WRITE_SIZE*1024 per launch (MI355X_MICROARCH.md gfx950 corrections); "
                     "fabric-side L2 counters, Infinity Cache hits included"}
        if "SQ_INSTS_VALU" in pmc:
            # wave-level VALU instructions per launch (each issues over 2 cycles on a SIMD-32: MI355X_MICROARCH.md)
            t["valu_insts_per_launch"] = pmc["SQ_INSTS_VALU"]
            if pmc.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in pmc:
                t["valu_lane_util"] = pmc["SQ_THREAD_CYCLES_VALU"] / (64.0 * pmc["SQ_ACTIVE_INST_VALU"])
        if "SQ_INSTS_VMEM_RD" in pmc:
            # wave-level vector-memory instructions per launch (bench.py roofline.vmem: against the TD unit's floor)
            t["vmem_rd_insts_per_launch"] = pmc["SQ_INSTS_VMEM_RD"]
            t["vmem_wr_insts_per_launch"] = pmc.get("SQ_INSTS_VMEM_WR")
            t["vmem_insts_per_launch"] = pmc["SQ_INSTS_VMEM_RD"] + pmc.get("SQ_INSTS_VMEM_WR", 0.0)
        if "wave_cycle_split" in k:
            t["wait_any_frac"] = k["wave_cycle_split"].get("wait_any")
        if "l2_hit_rate" in k:
            t["l2_hit_rate"] = k["l2_hit_rate"]
        if "vmem_unit_busy" in k:
            t["vmem_unit_busy"] = k["vmem_unit_busy"]
        (out / a.traffic_out).write_text(json.dumps(t, indent=1) + "\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
