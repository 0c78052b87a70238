#!/usr/bin/env python3
"""Render-server diagnostics (GPU): frames posted k per call through the server, against the batched launch, with a
short gate timeout (HALOGEN_SERVER_GATE_TIMEOUT_MS) so a lost frame is an error, not a hang.  Every call's time,
server launches / frames and the first frame count whose image differs are logged, line by line, to the file given.

  HALOGEN_SERVER_GATE_TIMEOUT_MS=2000 python3 tools/server_diag.py gpurun_out/r05b/diag.log [--check-every 8]"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "halogen-pathtracer_amd"), str(ROOT / "tests")]
import cases  # noqa: E402
from halogen import abi  # noqa: E402


def gpu_render(packed, params, frames, acc=True, cube=None, tiling=None):
    """The batched launch (one hg_render of `frames` frames: more than the server takes, so never through it)."""
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    with abi.Context(0) as ctx:
        ctx.set_option(abi.HG_OPT_SERVER, 0)
        ctx.upload_scene(packed)
        if cube is not None:
            ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
        ctx.resize(W, H)
        if tiling:
            ctx.set_tiling(*tiling)
        ctx.set_params(params)
        ctx.render(frames, acc)
        img = np.full((H, W, 4), np.nan, np.float32)
        ctx.readback(W, H, img)
        return img, ctx.counters()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--case", default="dragon10_64x36")
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--per-call", default="1,2,8")
    ap.add_argument("--check-every", type=int, default=0, help="read back and compare every k frames (0: at the end)")
    ap.add_argument("--tilings", default="none,2/3")
    ap.add_argument("--server", type=int, default=2, help="HG_OPT_SERVER (2: every qualifying call)")
    a = ap.parse_args()
    Path(a.log).parent.mkdir(parents=True, exist_ok=True)
    out = open(a.log, "w")

    def log(*x):
        out.write(" ".join(str(v) for v in x) + "\n")
        out.flush()

    packed, params, cube, _, _ = cases.setup(a.case)
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    for tl in a.tilings.split(","):
        tiling = None if tl == "none" else tuple(int(v) for v in tl.split("/"))
        checks = list(range(a.check_every, a.frames + 1, a.check_every)) if a.check_every else []
        if a.frames not in checks:
            checks.append(a.frames)
        refs = {k: gpu_render(packed, params, k, True, cube, tiling=tiling)[0] for k in checks}
        for per_call in (int(v) for v in a.per_call.split(",")):
            ctx = abi.Context(0)
            ctx.set_option(abi.HG_OPT_COALESCE, 1)
            ctx.set_option(abi.HG_OPT_SERVER, a.server)
            ctx.upload_scene(packed)
            if cube is not None:
                ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
            ctx.resize(W, H)
            if tiling:
                ctx.set_tiling(*tiling)
            ctx.set_params(params)
            done, first_bad, t_start = 0, None, time.perf_counter()
            try:
                while done < a.frames:
                    n = min(per_call, a.frames - done)
                    t0 = time.perf_counter()
                    ctx.render(n, True)
                    dt = time.perf_counter() - t0
                    done += n
                    if dt > 0.005:
                        log(f"  tiling {tiling} per_call {per_call}: call ending at frame {done} took {dt * 1e3:.1f} ms")
                    if done in refs:
                        img = np.full((H, W, 4), np.nan, np.float32)
                        ctx.readback(W, H, img)
                        c = ctx.counters()
                        bad = int((img.view(np.uint32) != refs[done].view(np.uint32)).sum())
                        log(f"  frame {done}: {bad} floats differ; server launches {c['server_launches']}, "
                            f"frames {c['server_frames']}")
                        if bad and first_bad is None:
                            first_bad = done
                log(f"tiling {tiling} per_call {per_call}: {a.frames} frames in {time.perf_counter() - t_start:.2f} s, "
                    f"first bad frame {first_bad}")
            except Exception as e:  # noqa: BLE001
                log(f"tiling {tiling} per_call {per_call}: ERROR at frame {done}: {e}")
            finally:
                log("closing")
                ctx.close()
                log("closed")


if __name__ == "__main__":
    main()
    print("diag: main returned", flush=True)
