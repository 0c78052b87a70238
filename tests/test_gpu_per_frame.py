"""The drop-in's operating point and its checkpoint state, through the C-ABI.

The reference dispatches HalogenCompute once per frame (RP:327, dispatch RP:406) and blends it into the accumulation
target (RP:343-347); hg_render(n) runs n such frames in one launch.  Launches of few frames take their own path through
the kernels (the streaming kernel's persistent work-queue form, the lean blend, the tile order re-sorted every
HG_ORDER_MIN_FRAMES frames per trace stream, traces of consecutive launches overlapping on two streams), and
consecutive hg_render calls are held and launched together (HG_OPT_COALESCE) until something observes the state; both
are checked bit for bit against the batched launch: strict (coalesce 1: every call its own launch) and coalesced.

Checkpoint/resume: the reference's resumable state is the accumulation target plus FrameCount (RP:152, 185, 347);
hg_readback exports it and hg_set_accumulation restores it into a fresh context."""
import json
from pathlib import Path

import numpy as np
import pytest

import cases
import hg_oracle
from halogen import abi, render_pass as rp, scenes
from test_gpu_parity import assert_bitwise, gpu_render

GOLD = Path(__file__).resolve().parent / "golden"


def _full(cfg_name):
    cfg = scenes.CONFIGS[cfg_name]
    settings = scenes.settings_for(cfg)
    s = rp.clamp_settings(settings)
    packed = cases._scene(cfg.scene, 10)
    cube = settings.environmentCubemap if s["UseEnvironmentCubemap"] else None
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), cube is not None)
    return packed, params, cube


@pytest.mark.gpu
@pytest.mark.parametrize("coalesce", [1, 3, 16])
@pytest.mark.parametrize("name", ["dragon10_64x36", "glass_64x36", "c1_64", "c1_48_noacc", "c1_64_spp3"])
def test_gpu_one_frame_launches_match_golden(gpu, name, coalesce):
    """frames x hg_render(1) (the reference's per-frame dispatches) equals the golden image and counters, and the
    batched hg_render(frames), for the streaming (dragon, Cornell) and regenerating (glass) kernels, without
    accumulation and with spp 3; every call its own launch (coalesce 1) or held 3 / 16 frames at a time."""
    meta = json.loads((GOLD / f"{name}.json").read_text())
    packed, params, cube, frames, acc = cases.setup(name)
    img, cnt = gpu_render(packed, params, frames, acc, cube, splits=[1] * frames, coalesce=coalesce)
    assert_bitwise(img, np.load(GOLD / f"{name}.npz")["image"], f"{name} as {frames} x render(1), coalesce {coalesce}")
    for k, v in meta["counters"].items():
        assert cnt[k] == v, (k, cnt[k], v)
    assert cnt["launches"] == -(-frames // coalesce)


@pytest.mark.gpu
def test_gpu_coalesced_frames_flush_at_every_observation(gpu):
    """Held frames are launched before anything reads or changes the context: a readback after 3 held calls is the
    3-frame image; a counters read, set_params with a new camera, clear_accumulation and set_accumulation all see the
    held frames first."""
    packed, params, cube, frames, acc = cases.setup("dragon10_64x36")
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    three, c3 = gpu_render(packed, params, 3, True, cube)
    five, _ = gpu_render(packed, params, 5, True, cube)
    with abi.Context(0) as ctx:
        ctx.set_option(abi.HG_OPT_COALESCE, 64)
        ctx.upload_scene(packed)
        ctx.resize(W, H)
        ctx.set_params(params)
        for _ in range(3):
            ctx.render(1, True)
        assert_bitwise(ctx.readback(W, H), three, "readback after 3 held frames")
        for _ in range(2):
            ctx.render(1, True)
        assert ctx.counters()["paths"] == c3["paths"] // 3 * 5  # the held frames ran before the read
        assert_bitwise(ctx.readback(W, H), five, "5 frames")
        ctx.render(1, True)
        ctx.clear_accumulation()  # launches the held frame first, then clears
        ctx.set_params(params)
        for _ in range(3):
            ctx.render(1, True)
        ctx.set_params(params)  # launches the 3 held frames (FrameCount 1..3), then resets FrameCount to 1
        assert_bitwise(ctx.readback(W, H), three, "held frames launched by set_params")
        ctx.render(2, True)
        ctx.set_accumulation(three, 4)  # the 2 held frames land first, then the checkpoint overwrites them
        ctx.render(2, True)
        assert_bitwise(ctx.readback(W, H), five, "checkpoint after held frames")


@pytest.mark.gpu
@pytest.mark.parametrize("cfg_name", ["C3", "C5", "C2"])
def test_gpu_one_frame_launches_match_batched_full_size(gpu, cfg_name):
    """BASELINE's C3 (871k dragon, streaming kernel), C5 (glass + cubemap, regenerating kernel) and C2 (Cornell box,
    streaming kernel on a shallow BVH) at 1920x1080:
    64 x hg_render(1) from a cleared accumulator is bit-identical to one hg_render(64) over the whole image, and a
    band of rows of it equals the live oracle."""
    packed, params, cube = _full(cfg_name)
    frames = 64
    batched, bc = gpu_render(packed, params, frames, True, cube)
    for coalesce in (1, 16):
        single, sc = gpu_render(packed, params, frames, True, cube, splits=[1] * frames, coalesce=coalesce)
        assert_bitwise(single, batched, f"{cfg_name}: 64 x render(1) vs render(64), coalesce {coalesce}")
        for k in ("paths", "rays", "tri_tests", "aabb_tests", "hits"):
            assert sc[k] == bc[k], (k, sc[k], bc[k])
    W = int(params.screenParameters.x)
    y0, y1 = 538, 540
    ref, _ = hg_oracle.render(packed, params, 2, True, cubemap=cube, pix_range=(y0 * W, y1 * W))
    two, _ = gpu_render(packed, params, 2, True, cube, splits=[1, 1], coalesce=1)
    assert_bitwise(two[y0:y1], ref[y0:y1], f"{cfg_name} rows {y0}-{y1}, 2 x render(1) vs oracle")


@pytest.mark.gpu
def test_gpu_share_holds_calls_until_it_fills_the_gpu(gpu):
    """A rank's 1/8 share of C3 (4,050 of 32,400 tiles) holds consecutive 64-frame calls until its launch has as many
    rounds of 64-frame tile waves as one context's whole image (HG_SHARE_HOLD_ROUNDS: 8 calls here), and runs one
    launch of split tile waves; every call its own launch (coalesce 1: the queue form) and one hg_render(512) give the
    same image, bit for bit."""
    packed, params, cube = _full("C3")
    held, hc = gpu_render(packed, params, 512, True, cube, tiling=(0, 8), splits=[64] * 8)
    strict, sc = gpu_render(packed, params, 512, True, cube, tiling=(0, 8), splits=[64] * 8, coalesce=1)
    one, _ = gpu_render(packed, params, 512, True, cube, tiling=(0, 8))
    assert hc["launches"] == 1 and sc["launches"] == 8, (hc["launches"], sc["launches"])
    assert_bitwise(held, strict, "1/8 share: 8 x render(64) held vs each launched")
    assert_bitwise(one, strict, "1/8 share: render(512) vs 8 x render(64)")
    assert hc["paths"] == sc["paths"]


@pytest.mark.gpu
def test_gpu_mixed_launch_sizes_with_tile_order(gpu):
    """1-frame launches between multi-frame ones, with the cost order re-sorted only every 16 frames and a rank's share
    of the tiles: the same image as one launch."""
    packed, params, cube, frames, acc = cases.setup("dragon10_64x36")
    for tiling in (None, (1, 3)):
        ref, _ = gpu_render(packed, params, 40, True, cube, tiling=tiling)
        for coalesce in (1, 4):
            img, _ = gpu_render(packed, params, 40, True, cube, tiling=tiling, splits=[1] * 17 + [5] + [1] * 18,
                                coalesce=coalesce)
            assert_bitwise(img, ref, f"mixed launches, tiling {tiling}, coalesce {coalesce}")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["dragon10_64x36", "glass_64x36", "c1_64_spp3"])
def test_gpu_checkpoint_resume_bit_identical(gpu, name):
    """render(16) -> hg_readback -> a NEW context -> hg_set_accumulation(image, FrameCount 17) -> render(16) equals
    render(32) bit for bit; also as one rank's share of a 3-way tiling."""
    packed, params, cube, frames, acc = cases.setup(name)
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    for tiling in (None, (2, 3)):
        ref, _ = gpu_render(packed, params, 32, True, cube, tiling=tiling)
        first, _ = gpu_render(packed, params, 16, True, cube, tiling=tiling)
        with abi.Context(0) as ctx:
            ctx.upload_scene(packed)
            if cube is not None:
                ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
            ctx.resize(W, H)
            if tiling:
                ctx.set_tiling(*tiling)
            ctx.set_params(params)  # frameCount 1: hg_set_accumulation below overrides it
            ctx.set_accumulation(np.nan_to_num(first, nan=0.0), 17)
            ctx.render(16, True)
            img = np.full((H, W, 4), np.nan, np.float32)
            ctx.readback(W, H, img)
        assert_bitwise(img, ref, f"{name} resumed at frame 17, tiling {tiling}")


@pytest.mark.gpu
def test_gpu_render_pass_restore(gpu):
    """HalogenRenderPass.restore(read_image(), getFrameCount()) on a new pass continues bit-identically."""
    cfg = scenes.CONFIGS["C1"].resized(40, 32, 3)
    scene = cfg.build_scene()
    cam = cfg.camera()
    a = rp.HalogenRenderPass(cfg.settings)
    for _ in range(6):
        a.Execute(scene, cam)
    want = a.read_image()
    b = rp.HalogenRenderPass(cfg.settings)
    for _ in range(3):
        b.Execute(scene, cam)
    state = (b.read_image(), b.getFrameCount())
    b.Dispose()
    c = rp.HalogenRenderPass(cfg.settings)
    c.restore(*state)
    for _ in range(3):
        c.Execute(scene, cam)
    assert c.getFrameCount() == a.getFrameCount() == 7
    assert_bitwise(c.read_image(), want, "render pass restore")
    a.Dispose()
    c.Dispose()


@pytest.mark.gpu
def test_gpu_set_accumulation_errors_are_loud(gpu):
    packed, params, cube, frames, acc = cases.setup("c1_64")
    with abi.Context(0) as ctx:
        with pytest.raises(abi.HalogenError, match="hg_resize not called"):
            ctx.set_accumulation(np.zeros((64, 64, 4), np.float32), 1)
        ctx.resize(64, 64)
        with pytest.raises(abi.HalogenError, match="too small"):
            ctx.set_accumulation(np.zeros((32, 64, 4), np.float32), 1)
        with pytest.raises(abi.HalogenError, match="frame_count"):
            ctx.set_accumulation(np.zeros((64, 64, 4), np.float32), 0)


@pytest.mark.gpu
def test_gpu_display_readback_pipelined(gpu):
    """hg_readback_begin/_end (the C# pass's display path): each frame's image equals the image of that many frames,
    when taken at once (begin, end) and one frame behind (two outstanding); with a 3-way tiling the other ranks'
    pixels read 0; misuse fails loudly; hg_resize drops the outstanding readbacks."""
    packed, params, cube, frames, acc = cases.setup("dragon10_64x36")
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    want = [gpu_render(packed, params, k, True, cube)[0] for k in (1, 2, 3, 4, 5)]
    with abi.Context(0) as ctx:
        ctx.upload_scene(packed)
        ctx.resize(W, H)
        with pytest.raises(abi.HalogenError, match="no readback outstanding"):
            ctx.readback_end(W, H)
        ctx.set_params(params)
        ctx.render(1, True)
        ctx.readback_begin()
        assert_bitwise(ctx.readback_end(W, H), want[0], "display readback, frame 1")
        got = []
        for k in range(1, 5):  # frames 2..5, one frame behind
            ctx.render(1, True)
            ctx.readback_begin()
            if k >= 2 and k < 4:
                got.append(ctx.readback_end(W, H))
        with pytest.raises(abi.HalogenError, match="2 readbacks outstanding"):  # frames 4 and 5 are
            ctx.readback_begin()
        got.append(ctx.readback_end(W, H))
        got.append(ctx.readback_end(W, H))
        for k, img in enumerate(got):
            assert_bitwise(img, want[k + 1], f"pipelined display readback, frame {k + 2}")
        with pytest.raises(abi.HalogenError, match="no readback outstanding"):
            ctx.readback_end(W, H)


@pytest.mark.gpu
def test_gpu_display_readback_tiling_and_resize(gpu):
    packed, params, cube, frames, acc = cases.setup("dragon10_64x36")
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    full, _ = gpu_render(packed, params, 2, True, cube)
    own, _ = gpu_render(packed, params, 2, True, cube, tiling=(1, 3))  # other ranks' pixels NaN (left untouched)
    with abi.Context(0) as ctx:
        ctx.upload_scene(packed)
        ctx.resize(W, H)
        ctx.set_tiling(1, 3)
        ctx.set_params(params)
        ctx.render(2, True)
        ctx.readback_begin()
        img = ctx.readback_end(W, H, copy=False)
        mine = ~np.isnan(own[..., 0])
        assert mine.any() and (~mine).any()
        assert_bitwise(img[mine], full[mine], "display readback, this rank's pixels")
        assert not img[~mine].any(), "other ranks' pixels must read 0"
        ctx.readback_begin()
        ctx.resize(W // 2, H)  # drops the outstanding readback (and its image)
        with pytest.raises(abi.HalogenError, match="no readback outstanding"):
            ctx.readback_end(W // 2, H)


@pytest.mark.gpu
@pytest.mark.parametrize("lane_pick", [0, 1])
def test_gpu_display_deep_ring(gpu, lane_pick):
    """Up to HG_READBACK_MAX (16) display readbacks outstanding, every call its own 1-frame launch, on the first idle
    trace stream (HG_OPT_LANE_PICK 1, the default) or on the streams in turn: each displayed image equals the image of
    that many frames."""
    assert abi.HG_READBACK_MAX == 16
    packed, params, cube, frames, acc = cases.setup("dragon10_64x36")
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    n = 20
    want = [gpu_render(packed, params, k, True, cube)[0] for k in range(1, n + 1)]
    with abi.Context(0) as ctx:
        ctx.set_option(abi.HG_OPT_LANE_PICK, lane_pick)
        ctx.set_option(abi.HG_OPT_COALESCE, 1)
        ctx.set_option(abi.HG_OPT_READBACK_DEPTH, 16)
        with pytest.raises(abi.HalogenError, match="readback depth"):
            ctx.set_option(abi.HG_OPT_READBACK_DEPTH, 17)
        ctx.upload_scene(packed)
        ctx.resize(W, H)
        ctx.set_params(params)
        got, pending = [], 0
        for _ in range(n):
            ctx.render(1, True)
            ctx.readback_begin()
            pending += 1
            if pending == 16:
                got.append(ctx.readback_end(W, H))
                pending -= 1
        while pending:
            got.append(ctx.readback_end(W, H))
            pending -= 1
        assert len(got) == n
        for k, img in enumerate(got):
            assert_bitwise(img, want[k], f"display ring of 16, frame {k + 1}, lane pick {lane_pick}")
