"""Pipelined launches whose last chunk is a single frame.

A regenerating launch on the trace pipeline (hg_runtime.hip render_now) is chunked at HG_REGEN_MAX_CHUNK frames, or at
fewer when the per-frame colour buffer would pass its 4 GiB cap (2048 x 2048: 64 MiB per frame -> 64-frame chunks).  With
a frame split of 3, a 65-frame launch is one 64-frame chunk split 3 ways and one 1-frame chunk, whose own split is 1.
Every chunk of a pipelined launch is blended in frame order afterwards, so every chunk must store its colours, the
1-frame tail included.  In the HG_REGEN_ITEMS=0 A/B build (make noitems) the kernel used to decide from the chunk's own
split and blended the tail straight into the accumulator, after which the blend applied a stale colour buffer on top.

test_gpu_pipelined_tail_chunk runs the case on the product build; test_gpu_regen_noitems_build runs the same test in a
child process against halogen/noitems/libhalogen_hip.so (HALOGEN_LIB).  The reference for both is the lockstep kernel of
the same build (bit-exact against the oracle and the goldens, tests/test_gpu_parity.py)."""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from halogen import abi, render_pass as rp, scenes

ROOT = Path(__file__).resolve().parents[1]
NOITEMS_LIB = ROOT / "halogen-pathtracer_amd" / "halogen" / "noitems" / "libhalogen_hip.so"


def _render(packed, params, W, H, frames, kernel, split=None):
    with abi.Context(0) as ctx:
        ctx.set_option(abi.HG_OPT_KERNEL, kernel)
        ctx.set_option(abi.HG_OPT_COALESCE, 1)
        if split:
            ctx.set_option(abi.HG_OPT_FRAME_SPLIT, split)
        ctx.upload_scene(packed)
        ctx.resize(W, H)
        ctx.set_params(params)
        ctx.render(frames, True)
        img = ctx.readback(W, H)
        cnt = ctx.counters()
        build = ctx.selftest(abi.HG_SELFTEST_BUILD)[0]
    return img, cnt, build


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_gpu_pipelined_tail_chunk(gpu):
    W = H = 2048  # 65,536 tiles x 1 KiB per frame: 4 GiB / 64 MiB -> chunks of 64 frames
    frames = 65
    cfg = scenes.CONFIGS["C1"].resized(W, H, frames)
    s = rp.clamp_settings(scenes.settings_for(cfg))
    packed = cfg.build_scene().pack()
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), False)
    img, cnt, build = _render(packed, params, W, H, frames, abi.HG_KERNEL_MEGA_REGEN, split=3)
    ref, rcnt, _ = _render(packed, params, W, H, frames, abi.HG_KERNEL_MEGA)
    if os.environ.get("HG_EXPECT_NOITEMS") == "1":
        assert build & abi.HG_BUILD_NO_REGEN_ITEMS, f"{abi.LIB_PATH} is not the HG_REGEN_ITEMS=0 build"
    assert cnt["last_kernel"] == abi.HG_KERNEL_MEGA_REGEN
    bad = int((img.view(np.uint32) != ref.view(np.uint32)).sum())
    assert bad == 0, f"{bad} floats differ from the lockstep kernel"
    for k in ("paths", "rays", "tri_tests", "aabb_tests", "hits"):
        assert cnt[k] == rcnt[k], (k, cnt[k], rcnt[k])


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpu_regen_noitems_build(gpu):
    assert NOITEMS_LIB.exists(), f"{NOITEMS_LIB} not built (make -C halogen-pathtracer_amd noitems)"
    env = dict(os.environ, HALOGEN_LIB=str(NOITEMS_LIB), HG_EXPECT_NOITEMS="1")
    cmd = [sys.executable, "-u", "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
           "tests/test_gpu_regen_noitems.py::test_gpu_pipelined_tail_chunk",
           "tests/test_gpu_parity.py::test_gpu_frame_splits_and_tiling"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=500)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0 and " passed" in r.stdout and " failed" not in r.stdout, tail
