#!/usr/bin/env python3
"""Soak of the render server's close handshake: one-frame posts that keep meeting a server that is
closing or gone.  Each round: HG_OPT_SERVER_IDLE_US in {0, 10, 30, 100}, `frames` one-frame calls with a random host
pause of 0-150 us before each (busy wait, so the posts land at every point of the waves' close: before the closing
word, between it and the read of the post word, after), then the readback, bit for bit against one batched launch of
the same frames; counts lifetimes, refused posts and lost frames.  Exits non-zero on any difference or lost frame.

  python3 tools/server_soak.py [--rounds 8] [--frames 1000] [--seed 1]"""
import argparse
import random
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "halogen-pathtracer_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402

import cases  # noqa: E402
from halogen import abi  # noqa: E402


def spin(us):
    t = time.perf_counter() + us * 1e-6
    while time.perf_counter() < t:
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    rng = random.Random(a.seed)
    packed, params, cube, _, _ = cases.setup("dragon10_64x36")
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)

    def context(opts=None):
        ctx = abi.Context(0)
        for k, v in (opts or {}).items():
            ctx.set_option(k, v)
        ctx.upload_scene(packed)
        if cube is not None:
            ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
        ctx.resize(W, H)
        ctx.set_params(params)
        return ctx

    with context() as ref_ctx:
        ref_ctx.render(a.frames, True)
        ref = ref_ctx.readback(W, H)
    bad = 0
    totals = {"server_launches": 0, "server_refused": 0, "frames_lost": 0, "server_frames": 0}
    for r in range(a.rounds):
        idle = [0, 10, 30, 100][r % 4]
        with context({abi.HG_OPT_SERVER: 2, abi.HG_OPT_COALESCE: 1, abi.HG_OPT_SERVER_IDLE_US: idle}) as ctx:
            t0 = time.perf_counter()
            for _ in range(a.frames):
                spin(rng.uniform(0.0, 150.0))
                ctx.render(1, True)
            img = ctx.readback(W, H)
            c = ctx.counters()
        same = np.array_equal(img.view(np.uint32), ref.view(np.uint32))
        bad += 0 if same and c["frames_lost"] == 0 and c["server_frames"] == a.frames else 1
        for k in totals:
            totals[k] += int(c[k])
        print(f"round {r}: idle {idle:3d} us, {a.frames} frames in {time.perf_counter() - t0:.2f} s: "
              f"{c['server_launches']} lifetimes, {c['server_refused']} refused posts, {c['frames_lost']} lost, "
              f"bit-identical {same}", flush=True)
    print(f"total: {a.rounds} rounds, {totals}, rounds failing: {bad}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
