#!/usr/bin/env python3
"""Timeline of the persistent queue waves of 1-frame launches (analysis build HG_WAVE_TIMELINE=1 under variants/):
for each of the last launches, when its waves started, when each found the queue dry, when it ended, relative to the
launch's first wave start — the ramp (start spread), the busy part (to the median dry time) and the drain (dry to end,
the slowest path in flight).  Modes: `sync` (one 1-frame launch at a time: render, wait), `strict` (64 launches back
to back), `display2` (one frame behind).
  HALOGEN_LIB=variants/lib_tl.so python tools/wave_timeline.py [sync strict display2]"""
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "halogen-pathtracer_amd")]
from halogen import abi, render_pass as rp, scenes  # noqa: E402

LAUNCHES, WAVES = 64, 8192


def stats(rec):
    """rec: (waves, 4) u64 of one launch -> ms figures (100-MHz ticks)"""
    rec = rec[rec[:, 0] > 0]
    if len(rec) == 0:
        return None
    t0 = rec[:, 0].min()
    s, d, e = (rec[:, 0] - t0) / 1e5, (np.where(rec[:, 1] > 0, rec[:, 1], rec[:, 2]) - t0) / 1e5, (rec[:, 2] - t0) / 1e5
    return {"waves": int(len(rec)), "start_p50": float(np.median(s)), "start_max": float(s.max()),
            "dry_p10": float(np.percentile(d, 10)), "dry_p50": float(np.median(d)), "dry_max": float(d.max()),
            "end_p50": float(np.median(e)), "end_p90": float(np.percentile(e, 90)), "end_max": float(e.max()),
            "drain_p50": float(np.median(e - d)), "drain_max": float((e - d).max()),
            "items_per_lane_mean": float(rec[:, 3].mean() / 64)}


def main():
    modes = sys.argv[1:] or ["sync", "strict", "display2"]
    L = abi.lib()
    fn = L.hg_debug_timeline
    fn.restype = C.c_int64
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    cfg = scenes.CONFIGS["C3"]
    s = rp.clamp_settings(scenes.settings_for(cfg))
    packed = cfg.build_scene().pack()
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), False)
    W, H = cfg.width, cfg.height
    for mode in modes:
        with abi.Context(0) as ctx:
            ctx.upload_scene(packed)
            ctx.resize(W, H)
            ctx.set_params(params)
            ctx.set_option(abi.HG_OPT_COALESCE, 1)
            for _ in range(32):  # warm-up: buffers, cost orders
                ctx.render(1, True)
            ctx.synchronize()
            ctx.clear_accumulation()
            ctx.set_params(params)
            t = time.perf_counter()
            if mode == "sync":
                for _ in range(LAUNCHES):
                    ctx.render(1, True)
                    ctx.synchronize()
            elif mode == "strict":
                for _ in range(LAUNCHES):
                    ctx.render(1, True)
            else:
                pending = 0
                for _ in range(LAUNCHES):
                    ctx.render(1, True)
                    ctx.readback_begin(abi.HG_DISPLAY_R11G11B10F)
                    pending += 1
                    if pending == 2:
                        ctx.readback_end(W, H, copy=False)
                        pending -= 1
                while pending:
                    ctx.readback_end(W, H, copy=False)
                    pending -= 1
            ctx.synchronize()
            dt = time.perf_counter() - t
            buf = np.zeros((LAUNCHES, WAVES, 4), np.uint64)
            n = fn(ctx._h, buf.ctypes.data, buf.nbytes)
            per = [stats(buf[i]) for i in range(LAUNCHES)]
            per = [p for p in per if p]
            keys = per[0].keys()
            mean = {k: float(np.mean([p[k] for p in per])) for k in keys}
            print(json.dumps({"mode": mode, "launches_recorded": int(n), "ms_per_frame": dt * 1e3 / LAUNCHES,
                              "mean_over_launches_ms": mean}), flush=True)


if __name__ == "__main__":
    main()
