"""The CPU oracle against its committed golden fixtures (tests/golden, made by tools/make_goldens.py) and
against itself (thread-count invariance, frame-split invariance, stage KATs)."""
import ctypes as C
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import cases
import hg_oracle

GOLD = Path(__file__).resolve().parent / "golden"


@pytest.mark.parametrize("name", sorted(cases.CASES))
def test_oracle_reproduces_golden(built, name):
    meta = json.loads((GOLD / f"{name}.json").read_text())
    packed, params, cube, frames, acc = cases.setup(name)
    assert cases.packed_digest(packed) == meta["scene_sha256"], "scene builder changed: regenerate goldens"
    img, cnt = hg_oracle.render(packed, params, frames, acc, cubemap=cube)
    assert hashlib.sha256(img.tobytes()).hexdigest() == meta["image_sha256"]
    for k, v in meta["counters"].items():
        assert cnt[k] == v, k


def test_thread_count_invariance(built):
    packed, params, cube, frames, acc = cases.setup("c1_64")
    a, ca = hg_oracle.render(packed, params, frames, acc, threads=1)
    b, cb = hg_oracle.render(packed, params, frames, acc, threads=7)
    assert np.array_equal(a, b) and ca == cb


def test_frame_split_invariance(built):
    """4 frames in one call == 2 + 2 (FrameCount continues): what hg_render(n) relies on."""
    packed, params, cube, frames, acc = cases.setup("c1_64")
    a, _ = hg_oracle.render(packed, params, 4, True)
    b, _ = hg_oracle.render(packed, params, 2, True)
    params.frameCount = 3
    b, _ = hg_oracle.render(packed, params, 2, True, acc=b)
    assert np.array_equal(a, b)


def test_first_frame_replaces_accumulator(built):
    """w = 1/FrameCount = 1 on frame 1: whatever was accumulated before is multiplied by 0."""
    packed, params, cube, frames, acc = cases.setup("c1_64")
    a, _ = hg_oracle.render(packed, params, 1, True)
    junk = np.full_like(a, 7.0)
    b, _ = hg_oracle.render(packed, params, 1, True, acc=junk)
    assert np.array_equal(a, b)
    assert np.all(a[..., 3] == 1.0)


def _f3(*v):
    return (C.c_float * 3)(*v)


def test_stage_kats(built):
    L = hg_oracle.lib()
    # sphere: unit sphere at z=5 from origin along +z hits at 4; from inside the far root
    assert L.hgo_sphere_t(_f3(0, 0, 0), _f3(0, 0, 1), _f3(0, 0, 5), 1.0) == 4.0
    assert L.hgo_sphere_t(_f3(0, 0, 5), _f3(0, 0, 1), _f3(0, 0, 5), 1.0) == 1.0
    # triangle: orientation +1 from the side cross(e1,e2) points to, -1 from behind; u/v/t exact here
    u, v, o = C.c_float(), C.c_float(), C.c_float()
    t = L.hgo_triangle_t(_f3(0.25, 0.25, 1), _f3(0, 0, -1), _f3(0, 0, 0), _f3(1, 0, 0), _f3(0, 1, 0),
                         C.byref(u), C.byref(v), C.byref(o))
    assert (t, u.value, v.value, o.value) == (1.0, 0.25, 0.25, 1.0)
    t = L.hgo_triangle_t(_f3(0.25, 0.25, -1), _f3(0, 0, 1), _f3(0, 0, 0), _f3(1, 0, 0), _f3(0, 1, 0),
                         C.byref(u), C.byref(v), C.byref(o))
    assert (t, o.value) == (1.0, -1.0)
    assert L.hgo_triangle_t(_f3(2, 2, 1), _f3(0, 0, -1), _f3(0, 0, 0), _f3(1, 0, 0), _f3(0, 1, 0),
                            None, None, None) == np.inf
    # AABB: returns tMin (negative inside), +inf on a miss; 1/0 = inf directions handled by minNum/maxNum
    inf = float("inf")
    assert L.hgo_aabb_t(_f3(-1, -1, -1), _f3(1, 1, 1), _f3(0, 0, -5), _f3(inf, inf, 1)) == 4.0
    assert L.hgo_aabb_t(_f3(-1, -1, -1), _f3(1, 1, 1), _f3(0, 0, 0), _f3(inf, inf, 1)) == -1.0
    assert L.hgo_aabb_t(_f3(-1, -1, -1), _f3(1, 1, 1), _f3(3, 0, -5), _f3(inf, inf, 1)) == inf


def test_reference_node_stack_never_overflows_c3(built):
    """The reference's BLAS stack is `int NodeStack[32]` (HC:397); 33 entries are possible in principle at the
    depth cap.  A band of the full C3 image (871k-triangle dragon) never needs more than 32 (the
    deepest over 16 full frames is 23), so the oracle's and the kernel's deeper stacks change no result there."""
    from halogen import render_pass as rp, scenes
    cfg = scenes.CONFIGS["C3"]
    s = rp.clamp_settings(scenes.settings_for(cfg))
    packed = cases._scene("dragon", 10)
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), False)
    hg_oracle.stack_stats(reset=True)
    _, cnt = hg_oracle.render(packed, params, 1, True, pix_range=(400 * cfg.width, 700 * cfg.width), stats=True)
    over, deepest = hg_oracle.stack_stats(reset=True)
    assert cnt["rays"] > 500_000
    assert over == 0 and 8 <= deepest <= 32, (over, deepest)


@pytest.mark.parametrize("name", ["c1_64", "dragon1_64x36", "glass_64x36"])
def test_stats_build_equals_plain_build(built, name):
    """The traversal diagnostics live only in the stats build (HGO_STATS=1, VERDICT r03 weak #3: a shared atomic in the
    plain build's traversal loop halved the CPU baseline).  Both builds give the same image bit for bit and the same
    counters; only the stats build collects visits and stack depths."""
    if name not in cases.CASES:
        pytest.skip(f"no case {name}")
    packed, params, cube, frames, acc = cases.setup(name)
    assert hg_oracle.lib().hgo_stats_build() == 0 and hg_oracle.lib(True).hgo_stats_build() == 1
    hg_oracle.visit_stats(reset=True)
    hg_oracle.stack_stats(reset=True)
    a, ca = hg_oracle.render(packed, params, frames, acc, cubemap=cube)
    assert hg_oracle.visit_stats()["inner"] == [0, 0, 0], "the plain build counted visits"
    b, cb = hg_oracle.render(packed, params, frames, acc, cubemap=cube, stats=True)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and ca == cb
    v = hg_oracle.visit_stats(reset=True)
    _, deepest = hg_oracle.stack_stats(reset=True)
    # every inner-node visit is counted once: 2 box tests per visit
    assert 2 * (sum(v["root"]) + sum(v["inner"])) == cb["aabb_tests"]
    assert deepest >= 1
