"""GPU parity: the HIP megakernel through the C-ABI against the committed golden fixtures and the live CPU
oracle.  The bar is bit-exact float32 equality (stronger than the 1e-4 relative bound of BASELINE.json's
north_star); integer work counters must match exactly."""
import json
import os
from pathlib import Path

import numpy as np
import pytest

import cases
import hg_oracle
from halogen import abi, render_pass as rp, scenes

GOLD = Path(__file__).resolve().parent / "golden"
REL_TOL = 1e-4  # north_star: "within 1e-4 relative fp32"; asserted only as a diagnostic, the test is bitwise


KERNELS = {"mega": abi.HG_KERNEL_MEGA, "regen": abi.HG_KERNEL_MEGA_REGEN, "stream": abi.HG_KERNEL_MEGA_STREAM,
           "auto": abi.HG_KERNEL_AUTO}


def gpu_render(packed, params, frames, acc=True, cube=None, tiling=None, ctx=None, splits=None, kernel="auto",
               block=None, coalesce=None):
    own = ctx is None
    ctx = ctx or abi.Context(0)
    ctx.set_option(abi.HG_OPT_KERNEL, KERNELS[kernel])
    if coalesce:
        ctx.set_option(abi.HG_OPT_COALESCE, coalesce)
    if block:
        ctx.set_option(abi.HG_OPT_BLOCK, block)
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    ctx.upload_scene(packed)
    if cube is not None:
        ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
    ctx.resize(W, H)
    if tiling:
        ctx.set_tiling(*tiling)
    ctx.set_params(params)
    for n in (splits or [frames]):
        ctx.render(n, acc)
    img = np.full((H, W, 4), np.nan, np.float32)
    ctx.readback(W, H, img)
    cnt = ctx.counters()
    if os.environ.get("HG_EXPECT_NO_EXEC_FALLBACK") == "1":  # tests/test_gpu_check_exec.py: an HG_CHECK_EXEC=1 build
        assert ctx.selftest(abi.HG_SELFTEST_BUILD)[0] & abi.HG_BUILD_CHECK_EXEC, f"{abi.LIB_PATH} is not a check build"
        assert cnt["exec_fallbacks"] == 0, f"leaf_dist ran under a partial EXEC {cnt['exec_fallbacks']} times"
        # the cost order of every sort was a permutation of the tiles (hg_order_verify)
        assert cnt["order_faults"] == 0, f"{cnt['order_faults']} cost-order placements out of range or repeated"
    if own:
        ctx.close()
    return img, cnt


def assert_bitwise(got, want, what=""):
    g, w = got.view(np.uint32), want.view(np.uint32)
    bad = g != w
    if bad.any():
        rel = np.abs(got.astype(np.float64) - want) / np.maximum(np.abs(want.astype(np.float64)), 1e-30)
        idx = np.argwhere(bad)[:5]
        pytest.fail(f"{what}: {int(bad.sum())} of {bad.size} floats differ (max rel {np.nanmax(rel):.3g}, "
                    f"first at {idx.tolist()}: got {got[tuple(idx[0])]} want {want[tuple(idx[0])]})")


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", sorted(KERNELS))
@pytest.mark.parametrize("name", sorted(cases.CASES))
def test_gpu_matches_golden(gpu, name, kernel):
    meta = json.loads((GOLD / f"{name}.json").read_text())
    packed, params, cube, frames, acc = cases.setup(name)
    assert cases.packed_digest(packed) == meta["scene_sha256"]
    img, cnt = gpu_render(packed, params, frames, acc, cube, kernel=kernel)
    assert_bitwise(img, np.load(GOLD / f"{name}.npz")["image"], name)
    for k, v in meta["counters"].items():
        assert cnt[k] == v, (k, cnt[k], v)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", sorted(KERNELS))
def test_gpu_frame_splits_and_tiling(gpu, kernel):
    packed, params, cube, frames, acc = cases.setup("c1_64")
    ref, _ = gpu_render(packed, params, 4, kernel=kernel)
    img, _ = gpu_render(packed, params, 4, splits=[1, 3], kernel=kernel)
    assert_bitwise(img, ref, "1+3 frames")
    for block in (64, 256):
        img, _ = gpu_render(packed, params, 4, kernel=kernel, block=block)
        assert_bitwise(img, ref, f"block {block}")
    for n_ranks in (2, 3, 8):
        parts = [gpu_render(packed, params, 4, tiling=(r, n_ranks), kernel=kernel)[0] for r in range(n_ranks)]
        merged = np.full_like(ref, np.nan)
        for p in parts:
            m = ~np.isnan(p)
            merged[m] = p[m]
        assert_bitwise(merged, ref, f"{n_ranks} tiles")


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", sorted(KERNELS))
@pytest.mark.parametrize("cfg_name,rows", [("C3", (536, 540)), ("C3", (300, 303)), ("C2", (536, 540)),
                                           ("C2", (760, 763)), ("C5", (400, 403)),
                                           ("C5", (500, 503))])
def test_gpu_full_size_rows_match_oracle(gpu, cfg_name, rows, kernel):
    """BASELINE-sized configs (1080p; C3 with the full 871,200-triangle dragon): a band of rows traced by the
    oracle must equal the same rows of the GPU image, bit for bit.  The bands cross the box (C2 760-763 also the
    ceiling light, seen directly by ~10 % of its pixels): more than half of their paths hit geometry, and some of
    their pixels are lit after 2 frames (at 1 spp most Cornell paths end black: the light is small)."""
    cfg = scenes.CONFIGS[cfg_name]
    settings = scenes.settings_for(cfg)
    s = rp.clamp_settings(settings)
    packed = cases._scene(cfg.scene, 10)
    cube = settings.environmentCubemap if s["UseEnvironmentCubemap"] else None
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), cube is not None)
    frames = 2
    img, _ = gpu_render(packed, params, frames, True, cube, kernel=kernel)
    W = cfg.width
    y0, y1 = rows
    ref, rcnt = hg_oracle.render(packed, params, frames, True, cubemap=cube, pix_range=(y0 * W, y1 * W))
    assert_bitwise(img[y0:y1], ref[y0:y1], f"{cfg_name} rows {rows}")
    assert np.all(img[..., 3] == 1.0) and np.isfinite(img).all()
    lit = (ref[y0:y1, :, :3].max(-1) > 0).mean()
    assert rcnt["hits"] > 0.5 * rcnt["paths"] and lit > 0.03, (
        f"band {rows}: {rcnt['hits']} hits for {rcnt['paths']} paths, {lit:.3f} lit: not a parity check")


@pytest.mark.gpu
def test_gpu_render_pass_api(gpu):
    """HalogenRenderPass (the reference API surface) over the C-ABI: Execute x3 == one 3-frame dispatch,
    a camera move resets FrameCount, MaxAccumulatedFrames stops accumulation."""
    cfg = scenes.CONFIGS["C1"].resized(40, 32, 3)
    scene = cfg.build_scene()
    cam = cfg.camera()
    p1 = rp.HalogenRenderPass(cfg.settings)
    for _ in range(3):
        p1.Execute(scene, cam)
    a = p1.read_image()
    assert p1.getFrameCount() == 4
    p2 = rp.HalogenRenderPass(cfg.settings)
    p2.Execute(scene, cam, n_frames=3)
    assert_bitwise(p2.read_image(), a, "render pass batching")
    moved = scenes.cornell_camera(40, 32)
    moved.transform.position_local = (moved.transform.position_local[0] + 0.1,) + moved.transform.position_local[1:]
    p2.Execute(scene, moved)
    assert p2.getFrameCount() == 2
    import dataclasses
    p3 = rp.HalogenRenderPass(dataclasses.replace(cfg.settings, UnlimitedSampling=False, MaxAccumulatedFrames=2))
    for _ in range(4):
        p3.Execute(scene, cam)
    assert p3.getFrameCount() == 3
    for p in (p1, p2, p3):
        p.Dispose()


@pytest.mark.gpu
def test_gpu_errors_are_loud(gpu):
    packed, params, cube, frames, acc = cases.setup("c1_64")
    with abi.Context(0) as ctx:
        with pytest.raises(abi.HalogenError, match="hg_upload_scene not called"):
            ctx.render(1)
        ctx.upload_scene(packed)
        ctx.resize(64, 64)
        params.bufferCounts.y = 99
        ctx.set_params(params)
        with pytest.raises(abi.HalogenError, match="bufferCounts"):
            ctx.render(1)
        with pytest.raises(abi.HalogenError):
            ctx.set_tiling(3, 2)


@pytest.mark.gpu
def test_gpu_regen_limits_fall_back_bit_exact(gpu):
    """maxBounces above the regenerating kernel's byte-packed limit (250) runs the lockstep megakernel: the image
    and the work counters still equal the oracle's, and equal a lockstep render."""
    import dataclasses
    cfg = scenes.CONFIGS["C1"].resized(24, 16, 2)
    settings = dataclasses.replace(scenes.settings_for(cfg), MaxBounces=300, DiffuseBounces=300, GlossyBounces=300)
    s = rp.clamp_settings(settings)
    packed = cases._scene("cornell", 10)
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), False)
    assert params.maxBounces == 300
    img, cnt = gpu_render(packed, params, 2, True, None, kernel="regen")
    ref, ref_cnt = hg_oracle.render(packed, params, 2, True)
    assert_bitwise(img, ref, "maxBounces 300")
    lock, _ = gpu_render(packed, params, 2, True, None, kernel="mega")
    assert_bitwise(img, lock, "regen fallback vs lockstep")
    for k in ("rays", "tri_tests", "aabb_tests", "hits"):
        assert cnt[k] == ref_cnt[k], (k, cnt[k], ref_cnt[k])


@pytest.mark.gpu
@pytest.mark.parametrize("split", [1, 3, 7])
def test_gpu_frame_parallel_split_bit_exact(gpu, split):
    """Frame-parallel split (several waves per tile on disjoint frame ranges, colours blended in frame order) gives
    the image and counters of the unsplit render; also with a first FrameCount > 1 and without accumulation."""
    for name, first in (("c1_64", 1), ("c1_64", 5), ("c1_48_noacc", 1), ("glass_64x36", 1)):
        packed, params, cube, frames, acc = cases.setup(name, first_frame=first)
        frames = 8
        refs = []
        for sp in (1, split):
            with abi.Context(0) as ctx:
                ctx.set_option(abi.HG_OPT_FRAME_SPLIT, sp)
                refs.append(gpu_render(packed, params, frames, acc, cube, ctx=ctx, kernel="regen"))
        assert_bitwise(refs[1][0], refs[0][0], f"{name} first={first} split {split}")
        for k in ("paths", "rays", "tri_tests", "aabb_tests", "hits"):
            assert refs[1][1][k] == refs[0][1][k], (k, refs[1][1][k], refs[0][1][k])
    ref, _ = hg_oracle.render(*cases.setup("c1_64")[:2], 8, True)
    with abi.Context(0) as ctx:
        ctx.set_option(abi.HG_OPT_FRAME_SPLIT, split)
        img, _ = gpu_render(*cases.setup("c1_64")[:2], 8, True, None, ctx=ctx, kernel="regen")
    assert_bitwise(img, ref, f"split {split} vs oracle")


@pytest.mark.gpu
@pytest.mark.parametrize("t", [1, 4, 63])
@pytest.mark.parametrize("kernel", ["regen", "mega"])
def test_gpu_relaxed_descent_bit_exact(gpu, t, kernel):
    """Leaving the descent loop with up to t lanes still descending (they pause while the others test their leaves)
    keeps every lane's step order: golden images and counters are unchanged (including the deep dragon BLAS)."""
    for name in ("c1_64", "dragon1_64x36", "glass_64x36", "c1_32_tritests"):
        meta = json.loads((GOLD / f"{name}.json").read_text())
        packed, params, cube, frames, acc = cases.setup(name)
        with abi.Context(0) as ctx:
            ctx.set_option(abi.HG_OPT_DESCENT_T, t)
            img, cnt = gpu_render(packed, params, frames, acc, cube, ctx=ctx, kernel=kernel)
        assert_bitwise(img, np.load(GOLD / f"{name}.npz")["image"], f"{name} descent_t={t}")
        for k, v in meta["counters"].items():
            assert cnt[k] == v, (name, k, cnt[k], v)


@pytest.mark.gpu
def test_gpu_auto_kernel_choice(gpu):
    """HG_KERNEL_AUTO (the default) runs the streaming kernel for deep BLAS (the 871k dragon) or scenes of 4 or
    more meshes (the Cornell box's 9) and the regenerating kernel for a few shallow meshes (the glass scene's 2); the
    debug views always run the lockstep kernel."""
    with abi.Context(0) as ctx:
        assert ctx.counters()["last_kernel"] == 0
    for name, want in (("c1_64", abi.HG_KERNEL_MEGA_STREAM), ("glass_64x36", abi.HG_KERNEL_MEGA_REGEN),
                       ("c1_32_normal", abi.HG_KERNEL_MEGA)):
        packed, params, cube, frames, acc = cases.setup(name)
        _, cnt = gpu_render(packed, params, frames, acc, cube, kernel="auto")
        assert cnt["last_kernel"] == want, (name, cnt["last_kernel"])
    cfg = scenes.CONFIGS["C3"].resized(64, 64, 1)
    packed = cases._scene("dragon", 10)
    s = rp.clamp_settings(scenes.settings_for(cfg))
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), False)
    _, cnt = gpu_render(packed, params, 2, True, None, kernel="auto")
    assert cnt["last_kernel"] == abi.HG_KERNEL_MEGA_STREAM


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["regen", "stream"])
@pytest.mark.parametrize("name", ["c1_64", "glass_64x36", "dragon1_64x36"])
def test_gpu_tile_order_bit_exact(gpu, name, kernel):
    """Cost-ordered dispatch (HG_OPT_TILE_ORDER): every launch after the first traces its tiles in the order of the
    previous launch's wave times.  Several render calls (so later launches use a recorded order), unsplit and split,
    whole image and one rank's share, give the image and counters of the tile-index order."""
    packed, params, cube, frames, acc = cases.setup(name)
    for tiling in (None, (1, 3)):
        for split in (1, 3):
            out = []
            for on in (0, 1):
                with abi.Context(0) as ctx:
                    ctx.set_option(abi.HG_OPT_TILE_ORDER, on)
                    ctx.set_option(abi.HG_OPT_FRAME_SPLIT, split)
                    out.append(gpu_render(packed, params, 8, acc, cube, tiling=tiling, ctx=ctx, splits=[1, 2, 3, 2],
                                          kernel=kernel))
            assert_bitwise(out[1][0], out[0][0], f"{name} {kernel} tiling {tiling} split {split}")
            for k in ("paths", "rays", "tri_tests", "aabb_tests", "hits"):
                assert out[1][1][k] == out[0][1][k], (k, out[1][1][k], out[0][1][k])
    if name == "c1_64":
        ref, _ = hg_oracle.render(packed, params, 8, acc)
        with abi.Context(0) as ctx:
            img, _ = gpu_render(packed, params, 8, acc, cube, ctx=ctx, splits=[2, 2, 4], kernel=kernel)
        assert_bitwise(img, ref, f"{kernel} ordered vs oracle")


@pytest.mark.gpu
def test_gpu_c4_tiles(gpu):
    """C4: the 871k dragon at 3840x2160 dealt in 8x8 tiles to 8 ranks (8 contexts on this GPU, one after another as
    the 8 GPUs of a node would run them), gathered with hg_comm (8-rank in-process transport) and compared with the
    oracle on row bands that include tile-row boundaries (1079|1080, 1591|1592) and the image's first/last rows."""
    cfg = scenes.CONFIGS["C4"]
    assert (cfg.width, cfg.height) == (3840, 2160)
    settings = scenes.settings_for(cfg)
    s = rp.clamp_settings(settings)
    packed = cases._scene(cfg.scene, 10)
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), False)
    W, H, n, frames = cfg.width, cfg.height, 8, 2
    ctxs = []
    try:
        for r in range(n):
            c = abi.Context(0)
            c.upload_scene(packed)
            c.resize(W, H)
            c.set_tiling(r, n)
            c.set_params(params)
            c.render(frames, True)
            c.synchronize()
            ctxs.append(c)
        with abi.Comm.all(ctxs) as comm:
            comm.gather(0)
            img = comm.readback(W, H)
    finally:
        for c in ctxs:
            c.close()
    assert np.all(img[..., 3] == 1.0) and np.isfinite(img).all()
    for y0, y1 in ((0, 2), (1078, 1082), (1590, 1594), (2158, 2160)):
        ref, _ = hg_oracle.render(packed, params, frames, True, pix_range=(y0 * W, y1 * W))
        assert_bitwise(img[y0:y1], ref[y0:y1], f"C4 rows {y0}-{y1}")
