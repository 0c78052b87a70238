"""The render server (HG_OPT_SERVER, csrc/hg_mega.hip kServer), through the C-ABI.  The tests
force it on (HG_OPT_SERVER 2: every qualifying call) except the one for the automatic choice (1, the default).

The reference dispatches HalogenCompute once per frame (RP:327, RP:406).  hg_render calls of few accumulating frames on
the streaming kernel post their frames to persistent trace waves that outlive the call; each frame's blend runs on the
context stream behind a gate on that frame's completion count.  Every image here is compared bit for bit with the
batched launch (or the committed golden and its counters), with the server off (every call its own launch), and across
every event that stops or restarts the server: a new camera, a checkpoint, a clear, counters, an idle gap, a launch of
another kind, readbacks in flight; posts racing the server's close handshake; and a lost frame (its gate gave up), which
must leave the accumulator as it was and make every readback report HG_E_FRAME_LOST until a clear."""
import json
import time
from pathlib import Path

import numpy as np
import pytest

import cases
from halogen import abi, render_pass as rp, scenes
from test_gpu_parity import assert_bitwise, gpu_render

GOLD = Path(__file__).resolve().parent / "golden"


def _ctx(packed, params, cube=None, server=2, coalesce=1, tiling=None, idle_us=None):
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    ctx = abi.Context(0)
    ctx.set_option(abi.HG_OPT_SERVER, server)
    if idle_us is not None:
        ctx.set_option(abi.HG_OPT_SERVER_IDLE_US, idle_us)
    ctx.set_option(abi.HG_OPT_COALESCE, coalesce)
    ctx.upload_scene(packed)
    if cube is not None:
        ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
    ctx.resize(W, H)
    if tiling:
        ctx.set_tiling(*tiling)
    ctx.set_params(params)
    return ctx, W, H


def _sized(cfg_name, w, h, frames=1):
    cfg = scenes.CONFIGS[cfg_name].resized(w, h, frames)
    settings = scenes.settings_for(cfg)
    packed = cases._scene(cfg.scene, 10)
    s = rp.clamp_settings(settings)
    cube = settings.environmentCubemap if s["UseEnvironmentCubemap"] else None
    return packed, rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), cube is not None), cube


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["dragon10_64x36", "c1_64", "c1_64_spp3"])
def test_gpu_server_one_frame_calls_match_golden(gpu, name):
    """frames x hg_render(1) through one server lifetime: the golden image and its counters (the server's waves count
    every ray, triangle and box test as the per-launch kernels do), one server launch, every frame posted."""
    meta = json.loads((GOLD / f"{name}.json").read_text())
    packed, params, cube, frames, acc = cases.setup(name)
    ctx, W, H = _ctx(packed, params, cube)
    with ctx:
        for _ in range(frames):
            ctx.render(1, True)
        img = ctx.readback(W, H)
        cnt = ctx.counters()
    assert_bitwise(img, np.load(GOLD / f"{name}.npz")["image"], f"{name}: {frames} frames through the server")
    for k, v in meta["counters"].items():
        assert cnt[k] == v, (k, cnt[k], v)
    assert cnt["server_launches"] == 1 and cnt["server_frames"] == frames, cnt


@pytest.mark.gpu
def test_gpu_server_off_launches_per_call(gpu):
    """HG_OPT_SERVER 0: every call its own launch (the round-4 pipeline), the same image; no server launched."""
    packed, params, cube, frames, acc = cases.setup("dragon10_64x36")
    ref, _ = gpu_render(packed, params, frames, True, cube)
    ctx, W, H = _ctx(packed, params, cube, server=0)
    with ctx:
        for _ in range(frames):
            ctx.render(1, True)
        img = ctx.readback(W, H)
        cnt = ctx.counters()
    assert_bitwise(img, ref, "server off")
    assert cnt["server_launches"] == 0 and cnt["launches"] == frames


@pytest.mark.gpu
@pytest.mark.parametrize("frames", [3, 40, 200])
def test_gpu_server_many_frames_match_batched(gpu, frames):
    """More frames than the colour ring (16) and the per-wave frame window (4) hold, posted one per call, in pairs and
    in eights (hg_render(n <= 8) posts n frames), as one rank's share of a 3-way tiling too: the batched image."""
    packed, params, cube, _, _ = cases.setup("dragon10_64x36")
    for tiling in (None, (2, 3)):
        ref, rc = gpu_render(packed, params, frames, True, cube, tiling=tiling)
        for per_call in (1, 2, 8):
            ctx, W, H = _ctx(packed, params, cube, tiling=tiling)
            with ctx:
                done = 0
                while done < frames:
                    n = min(per_call, frames - done)
                    ctx.render(n, True)
                    done += n
                img = np.full((H, W, 4), np.nan, np.float32)
                ctx.readback(W, H, img)
                cnt = ctx.counters()
            assert_bitwise(img, ref, f"{frames} frames, {per_call} per call, tiling {tiling}, "
                                     f"{cnt['server_launches']} server launches")
            assert cnt["server_frames"] == frames and cnt["paths"] == rc["paths"], cnt


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [1, 2, 4])
def test_gpu_server_display_readback(gpu, depth):
    """The C# pass's per-frame display: render(1), readback_begin, and readback_end once `depth` are outstanding (0, 1
    and 3 frames behind).  Each displayed image (R11G11B10F and RGBA32F) equals that many frames' image; the server
    serves every frame of the run (one launch)."""
    packed, params, cube, _, _ = cases.setup("dragon10_64x36")
    n = 12
    want = [gpu_render(packed, params, k, True, cube)[0] for k in range(1, n + 1)]
    for fmt in (abi.HG_DISPLAY_RGBA32F, abi.HG_DISPLAY_R11G11B10F):
        ctx, W, H = _ctx(packed, params, cube)
        with ctx:
            ctx.set_option(abi.HG_OPT_READBACK_DEPTH, depth)
            got, pending = [], 0
            for _ in range(n):
                ctx.render(1, True)
                ctx.readback_begin(fmt)
                pending += 1
                if pending == depth:
                    got.append(ctx.readback_end(W, H))
                    pending -= 1
            while pending:
                got.append(ctx.readback_end(W, H))
                pending -= 1
            cnt = ctx.counters()
        for k, img in enumerate(got):
            exp = want[k] if fmt == abi.HG_DISPLAY_RGBA32F else abi.pack_display(want[k], fmt)
            assert np.array_equal(np.asarray(img).view(np.uint8), np.asarray(exp).view(np.uint8)), \
                f"display depth {depth}, format {fmt}, frame {k + 1}"
        assert cnt["server_launches"] == 1 and cnt["server_frames"] == n, cnt


@pytest.mark.gpu
def test_gpu_server_restarts_keep_the_image(gpu):
    """Every event that ends a server lifetime, mid-run, against the same call sequence with the server off: a camera
    move (set_params with a new camera and FrameCount 1, then clear, as ClearAccumulation does, RP:262-268), a
    checkpoint (set_accumulation), a clear alone (the server keeps running: the clear is ordered between blends), a
    counters read, a launch of another kind (a 16-frame call), short idle gaps (the server stays), an idle gap longer
    than the server's idle time (it closes itself; the next post restarts it), an upload."""
    on, con = _restart_sequence(2)
    off, coff = _restart_sequence(0)
    for k, (a, b) in enumerate(zip(on, off)):
        assert_bitwise(a, b, f"server restarts, readback {k}")
    assert con["server_launches"] >= 6 and coff["server_launches"] == 0, (con, coff)
    for k in ("paths", "rays", "tri_tests", "aabb_tests", "hits"):
        assert con[k] == coff[k], (k, con[k], coff[k])


def _restart_sequence(server, options=()):
    """The call sequence of test_gpu_server_restarts_keep_the_image: its readbacks and the counters."""
    packed, params, cube, _, _ = cases.setup("dragon10_64x36")
    moved = cases.setup("dragon10_64x36")[1]
    moved.camLocalToWorld.m[12] += 0.05

    def run(server):
        ctx, W, H = _ctx(packed, params, cube, server=server)
        for opt, v in options:
            ctx.set_option(opt, v)
        imgs = []
        with ctx:
            def frames(k):
                for _ in range(k):
                    ctx.render(1, True)
                imgs.append(ctx.readback(W, H))
            frames(5)
            ctx.set_params(moved)
            ctx.clear_accumulation()
            frames(4)
            ctx.set_accumulation(imgs[0], 6)
            frames(3)
            ctx.clear_accumulation()
            frames(3)
            ctx.counters()
            frames(2)
            ctx.render(16, True)
            frames(2)
            time.sleep(0.08)
            frames(2)
            for _ in range(3):  # short idle gaps: the server stays (its ring-slot counts not zero)
                time.sleep(0.03)
                frames(3)
            time.sleep(0.3)  # past HG_OPT_SERVER_IDLE_US (200 ms): the server has closed itself
            frames(2)
            ctx.upload_scene(packed)
            frames(2)
            cnt = ctx.counters()
        return imgs, cnt

    return run(server)


@pytest.mark.gpu
def test_gpu_server_edge_tiles_and_small_images(gpu):
    """Images whose size is not a multiple of 8 (edge tiles of fewer than 64 pixels), a single tile (8x8: one unit per
    frame, fewer units than the server has waves), and a power-of-two tile count (the unit -> frame shift)."""
    for w, h in ((61, 35), (8, 8), (64, 64)):
        packed, params, cube = _sized("C3", w, h)
        ref, _ = gpu_render(packed, params, 24, True, cube)
        ctx, W, H = _ctx(packed, params, cube)
        with ctx:
            for _ in range(24):
                ctx.render(1, True)
            img = ctx.readback(W, H)
            cnt = ctx.counters()
        assert_bitwise(img, ref, f"{w}x{h} through the server")
        assert cnt["server_launches"] == 1, cnt


@pytest.mark.gpu
def test_gpu_server_full_size_c3_with_display(gpu):
    """BASELINE's C3 at 1920x1080: 64 x (render(1) + R11G11B10F display one frame behind) through one server lifetime
    is bit-identical to hg_render(64), and every displayed image is the host packing of that frame's fp32 image (checked
    for the last two, the rest against the batched images of a few frame counts)."""
    cfg = scenes.CONFIGS["C3"]
    packed, params, cube = _sized("C3", cfg.width, cfg.height)
    W, H = cfg.width, cfg.height
    checks = {1, 2, 17, 63, 64}
    want = {k: gpu_render(packed, params, k, True, cube)[0] for k in checks}
    ctx, _, _ = _ctx(packed, params, cube)
    with ctx:
        ctx.set_option(abi.HG_OPT_READBACK_DEPTH, 2)
        shown, pending = [], 0
        for _ in range(64):
            ctx.render(1, True)
            ctx.readback_begin(abi.HG_DISPLAY_R11G11B10F)
            pending += 1
            if pending == 2:
                shown.append(ctx.readback_end(W, H))
                pending -= 1
        shown.append(ctx.readback_end(W, H))
        img = ctx.readback(W, H)
        cnt = ctx.counters()
    assert_bitwise(img, want[64], "C3 1080p, 64 frames through the server")
    for k in checks:
        assert np.array_equal(shown[k - 1], abi.pack_display(want[k], abi.HG_DISPLAY_R11G11B10F)), f"displayed frame {k}"
    # one lifetime: whether a post is taken depends on no host clock (the close handshake), and no gap here reaches the
    # server's 200-ms idle time
    assert cnt["server_launches"] == 1 and cnt["server_frames"] == 64, cnt


@pytest.mark.gpu
def test_gpu_server_automatic_engages_only_ahead(gpu):
    """HG_OPT_SERVER 1 (the default): a host that queues one-frame calls (C3 1080p, no readback between them) runs
    ahead of the GPU and gets the server; a host that reads every frame back before the next call (the reference's
    display) never runs ahead and launches per call.  Both images equal the batched launch bit for bit."""
    cfg = scenes.CONFIGS["C3"]
    packed, params, cube = _sized("C3", cfg.width, cfg.height)
    W, H = cfg.width, cfg.height
    want = gpu_render(packed, params, 24, True, cube)[0]
    for display in (False, True):
        ctx, _, _ = _ctx(packed, params, cube, server=1)
        with ctx:
            for _ in range(24):
                ctx.render(1, True)
                if display:
                    ctx.readback_begin(abi.HG_DISPLAY_R11G11B10F)
                    ctx.readback_end(W, H)
            img = ctx.readback(W, H)
            cnt = ctx.counters()
        assert_bitwise(img, want, f"automatic server, display {display}")
        if display:
            assert cnt["server_launches"] == 0, cnt
        else:
            assert cnt["server_launches"] >= 1 and cnt["server_frames"] >= 16, cnt


@pytest.mark.gpu
@pytest.mark.parametrize("idle_us", [0, 30])
def test_gpu_server_posts_racing_the_close_handshake(gpu, idle_us):
    """HG_OPT_SERVER_IDLE_US 0 / 30: the server closes itself (sv_close) whenever it has nothing new for that long, so
    nearly every one-frame post of this small image meets a server that is closing or gone.  A post the closing wave
    did not read is refused and re-posted to a new lifetime (hg_counters.server_refused); one it did read is traced
    before the waves leave.  200 frames, one per call and in fours, equal the batched launch bit for bit, and no frame
    is lost (a lost one would make the readback fail with HG_E_FRAME_LOST)."""
    packed, params, cube, _, _ = cases.setup("dragon10_64x36")
    frames = 200
    ref, rc = gpu_render(packed, params, frames, True, cube)
    for per_call in (1, 4):
        ctx, W, H = _ctx(packed, params, cube, idle_us=idle_us)
        with ctx:
            for _ in range(frames // per_call):
                ctx.render(per_call, True)
            img = ctx.readback(W, H)
            cnt = ctx.counters()
        assert_bitwise(img, ref, f"idle {idle_us} us, {per_call} per call: {cnt['server_launches']} lifetimes, "
                                 f"{cnt['server_refused']} posts refused")
        assert cnt["server_frames"] == frames and cnt["frames_lost"] == 0 and cnt["paths"] == rc["paths"], cnt
        if idle_us == 0:  # (at 30 us the host's posts may all come sooner than that: no close is guaranteed)
            assert cnt["server_launches"] > 1, cnt  # the server closed between posts at least once
        print(f"idle {idle_us} us, {per_call} per call: {cnt['server_launches']} lifetimes, "
              f"{cnt['server_refused']} refused posts")


@pytest.mark.gpu
@pytest.mark.parametrize("tiling", [None, (1, 2)])
def test_gpu_server_lost_frame_leaves_the_accumulator(gpu, tiling):
    """A frame whose gate gives up (HG_OPT_SERVER_GATE_US 0: the gate of a 1080p C3 frame, launched microseconds after
    its post, finds the frame unfinished) is lost: its blend and every later one are skipped, so the accumulator keeps
    the image of the frames before it; hg_render refuses, and every readback (single-rank, a rank's tiles, the display
    ring) hands out that image with HG_E_FRAME_LOST, until hg_clear_accumulation starts a valid accumulation again."""
    cfg = scenes.CONFIGS["C3"]
    packed, params, cube = _sized("C3", cfg.width, cfg.height)
    W, H = cfg.width, cfg.height
    want3 = gpu_render(packed, params, 3, True, cube, tiling=tiling)[0]
    ctx, _, _ = _ctx(packed, params, cube, tiling=tiling)
    with ctx:
        for _ in range(3):
            ctx.render(1, True)
        before = np.full((H, W, 4), np.nan, np.float32)  # (with tiling, other ranks' pixels stay untouched)
        ctx.readback(W, H, before)
        assert_bitwise(before, want3, "3 frames before the loss")
        ctx.set_option(abi.HG_OPT_SERVER_GATE_US, 0)
        try:
            for _ in range(2):
                ctx.render(1, True)
        except abi.HalogenError as e:  # (the second call may already see the first frame's loss)
            assert e.rc == abi.HG_E_FRAME_LOST, e
        img = np.full((H, W, 4), np.nan, np.float32)
        with pytest.raises(abi.HalogenError) as e:
            ctx.readback(W, H, img)
        assert e.value.rc == abi.HG_E_FRAME_LOST, e.value
        assert_bitwise(img, before, "the accumulator after a lost frame")
        with pytest.raises(abi.HalogenError) as e:
            ctx.render(1, True)
        assert e.value.rc == abi.HG_E_FRAME_LOST
        ctx.readback_begin(abi.HG_DISPLAY_RGBA32F)
        with pytest.raises(abi.HalogenError) as e:
            ctx.readback_end(W, H)
        assert e.value.rc == abi.HG_E_FRAME_LOST
        cnt = ctx.counters()
        assert cnt["frames_lost"] >= 1, cnt
        # a clear starts a valid accumulation: the same 3 frames again (FrameCount 1) equal the batched image
        ctx.set_option(abi.HG_OPT_SERVER_GATE_US, -1)
        ctx.clear_accumulation()
        ctx.set_params(params)
        for _ in range(3):
            ctx.render(1, True)
        again = np.full((H, W, 4), np.nan, np.float32)
        ctx.readback(W, H, again)
    assert_bitwise(again, want3, "3 frames after the clear")


@pytest.mark.gpu
@pytest.mark.parametrize("ahead", [1, 2, 4])
def test_gpu_server_traces_ahead_keeps_the_image(gpu, ahead):
    """HG_OPT_SERVER_AHEAD with the counters off: the server traces `ahead` frames beyond the host's calls and blends
    a frame only when it is asked for.  The restart sequence (camera moves, checkpoint, clears, counters, a 16-frame
    launch, idle gaps, an upload: each abandons the frames traced ahead) gives the readbacks of the server off, bit for
    bit; so does a per-frame display at once and one frame behind, in the automatic mode (HG_OPT_SERVER 1), where the
    call chain engages the server although the host never runs ahead."""
    opts = ((abi.HG_OPT_COUNTERS, 0), (abi.HG_OPT_SERVER_AHEAD, ahead))
    on, con = _restart_sequence(2, opts)
    off, _ = _restart_sequence(0, opts)
    for k, (a, b) in enumerate(zip(on, off)):
        assert_bitwise(a, b, f"ahead {ahead}: server restarts, readback {k}")
    assert con["server_ahead"] > 0 and con["frames_lost"] == 0, con
    packed, params, cube, _, _ = cases.setup("dragon10_64x36")
    n = 12
    want = [gpu_render(packed, params, k, True, cube)[0] for k in range(1, n + 1)]
    for depth in (1, 2):
        ctx, W, H = _ctx(packed, params, cube, server=1)
        with ctx:
            for opt, v in opts:
                ctx.set_option(opt, v)
            ctx.set_option(abi.HG_OPT_READBACK_DEPTH, depth)
            got, pending = [], 0
            for _ in range(n):
                ctx.render(1, True)
                ctx.readback_begin(abi.HG_DISPLAY_RGBA32F)
                pending += 1
                if pending == depth:
                    got.append(ctx.readback_end(W, H))
                    pending -= 1
            while pending:
                got.append(ctx.readback_end(W, H))
                pending -= 1
            cnt = ctx.counters()
        for k, img in enumerate(got):
            assert_bitwise(img, want[k], f"ahead {ahead}, display depth {depth}, frame {k + 1}")
        assert cnt["server_launches"] >= 1 and cnt["server_frames"] >= n - 1 and cnt["server_ahead"] > 0, cnt
