#!/usr/bin/env python3
"""Per-instruction attribution of the texture-data unit's time (tools/pmc_attrib.sh output).

  python3 tools/pmc_attrib.py gpurun_out/prof/attrib_<TAG> [--json profiles/<TAG>_attrib.json]

Per launch of the timed trace kernel (the counter-free streaming kernel), per config: wave-level vector-memory
instructions (TD_LOAD_WAVEFRONT, cross-checked against SQ_INSTS_VMEM_RD + _WR), and per instruction the TD unit's busy
cycles split into waiting for L1 data (TD_TC_STALL) and the rest, the L1 tag lookups (TCP_TOTAL_CACHE_ACCESSES) and
misses to L2 (TCP_TCC_READ_REQ), and the L1's own stall causes.  GRBM_GUI_ACTIVE sums the 8 XCDs' clocks; TD / TCP
counters sum over the 256 CUs."""
import argparse
import collections
import csv
import glob
import json
import os

N_XCD, N_CU = 8, 256


def per_launch(d, kernel):
    tot, disp = collections.defaultdict(float), collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    return {k: tot[k] / len(disp[k]) for k in tot}


def attribute(p):
    w = p["TD_LOAD_WAVEFRONT_sum"]
    cyc = p["GRBM_GUI_ACTIVE"] / N_XCD
    busy, stall = p["TD_TD_BUSY_sum"], p["TD_TC_STALL_sum"]
    tags, miss = p["TCP_TOTAL_CACHE_ACCESSES_sum"], p["TCP_TCC_READ_REQ_sum"]
    out = {
        "vmem_wave_instructions": w,
        "sq_vmem_instructions": p.get("SQ_INSTS_VMEM_RD", 0) + p.get("SQ_INSTS_VMEM_WR", 0),
        "coalescable_share": p.get("TD_COALESCABLE_WAVEFRONT_sum", 0) / w,
        "kernel_cycles": cyc,
        "td_busy_frac": busy / (N_CU * cyc),
        "per_instruction": {
            "td_busy_cycles": busy / w,
            "td_waiting_on_l1_cycles": stall / w,
            "td_other_cycles": (busy - stall) / w,
            "l1_tag_lookups": tags / w,
            "l1_misses": miss / w,
            "tcp_wave_latency_cycles": p.get("TCP_TCP_LATENCY_sum", 0) / w,
            "tcp_pending_l2_stall_cycles": p.get("TCP_PENDING_STALL_CYCLES_sum", 0) / w,
            "tcp_tag_conflict_stall_cycles": p.get("TCP_READ_TAGCONFLICT_STALL_CYCLES_sum", 0) / w,
            "tcp_stalls_ta_data_cycles": p.get("TCP_TCP_TA_DATA_STALL_CYCLES_sum", 0) / w,
            "td_stalls_tcp_cycles": p.get("TCP_TD_TCP_STALL_CYCLES_sum", 0) / w,
            "tcr_stalls_tcp_cycles": p.get("TCP_TCR_TCP_STALL_CYCLES_sum", 0) / w,
            "lfifo_full_cycles": p.get("TCP_LFIFO_STALL_CYCLES_sum", 0) / w,
            "rfifo_full_cycles": p.get("TCP_RFIFO_STALL_CYCLES_sum", 0) / w,
            "ta_data_stalled_by_tc_cycles": p.get("TA_DATA_STALLED_BY_TC_CYCLES_sum", 0) / w,
            "ta_addr_stalled_by_td_cycles": p.get("TA_ADDR_STALLED_BY_TD_CYCLES_sum", 0) / w,
        },
        "l1_hit_rate": 1.0 - miss / max(tags, 1.0),
        "l2_read_latency_cycles": p.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / max(miss, 1.0),
        "lane_reads_per_instruction": p.get("TCP_TOTAL_READ_sum", 0) / w,
        "vmem_issue_level": p.get("SQ_INST_LEVEL_VMEM", 0) / max(p.get("SQ_ACTIVE_INST_VMEM", 0), 1.0),
        "wave_wait_inst_frac": p.get("SQ_WAIT_INST_ANY", 0) / max(p.get("SQ_WAVE_CYCLES", 0), 1.0),
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="hg_trace_stream_kernel<false")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    res = {}
    cfgs = sorted({os.path.basename(x).split("_p")[0] for x in glob.glob(os.path.join(a.dir, "*_p*")) if os.path.isdir(x)})
    for cfg in cfgs:
        p = {}
        for d in sorted(glob.glob(os.path.join(a.dir, f"{cfg}_p*"))):
            if os.path.isdir(d):
                p.update(per_launch(d, a.kernel))
        res[cfg] = {"per_launch": p, "attribution": attribute(p)}
    for cfg, r in res.items():
        print(f"== {cfg}")
        for k, v in r["attribution"].items():
            if isinstance(v, dict):
                for kk, vv in v.items():
                    print(f"  per instruction {kk:36s} {vv:10.3f}")
            else:
                print(f"  {k:52s} {v:14.6g}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
