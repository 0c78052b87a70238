"""Display readback in the display formats (hg_readback_begin_format / hg_readback_end_data, HG_OPT_READBACK_DEPTH;
VERDICT r03 missing #4).  The device packs the untiled accumulation target; the image must equal the host packing
(hg_pack_display, itself checked against independent restatements in tests/test_display_pack.py) of the RGBA32F readback
of the same frames, bit for bit, for every format, taken at once and several frames behind, and the accumulation target
must be untouched (the RGBA32F image after the packed readbacks equals the golden-path render).  Parity with D3D's own
R11G11B10 converter is unpinned (hg_pack.h)."""
import numpy as np
import pytest

import cases
from halogen import abi
from test_gpu_parity import assert_bitwise, gpu_render

FORMATS = [abi.HG_DISPLAY_RGBA32F, abi.HG_DISPLAY_RGBA16F, abi.HG_DISPLAY_R11G11B10F]


def _bits(a):
    return a.view(np.uint32) if a.dtype == np.float32 else a.view(np.uint16) if a.dtype == np.float16 else a


@pytest.mark.gpu
@pytest.mark.parametrize("side", [0, 1, 2])
@pytest.mark.parametrize("fmt", FORMATS)
def test_gpu_display_format_equals_host_packing(gpu, fmt, side):
    packed, params, cube, frames, acc = cases.setup("glass_64x36")  # emissive + sky: values above 1 and tiny ones
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    want = [gpu_render(packed, params, k, True, cube)[0] for k in (1, 2, 3, 4, 5, 6)]
    with abi.Context(0) as ctx:
        ctx.upload_scene(packed)
        if cube is not None:
            ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
        ctx.resize(W, H)
        ctx.set_params(params)
        ctx.set_option(abi.HG_OPT_READBACK_STREAM, side)  # copies on the context or side stream, or zero copy
        ctx.render(1, True)
        ctx.readback_begin(fmt)
        got = [ctx.readback_end(W, H)]  # frame 1, at once
        ctx.set_option(abi.HG_OPT_READBACK_DEPTH, 4)  # up to four outstanding: three frames behind
        pending = 0
        for _ in range(5):  # frames 2..6; frames 2 and 3 are taken when the fourth readback is in flight
            ctx.render(1, True)
            ctx.readback_begin(fmt)
            pending += 1
            if pending == 4:
                got.append(ctx.readback_end(W, H))
                pending -= 1
        ctx.readback_begin(fmt)  # frame 6 once more: four outstanding (frames 4, 5, 6, 6)
        pending += 1
        with pytest.raises(abi.HalogenError, match="4 readbacks outstanding"):
            ctx.readback_begin(fmt)
        if fmt != abi.HG_DISPLAY_RGBA32F:
            with pytest.raises(abi.HalogenError, match="hg_readback_end_data"):  # the float-only entry point refuses
                ptr = abi.C.POINTER(abi.C.c_float)()
                ctx._check(abi.lib().hg_readback_end(ctx._h, abi.C.byref(ptr), None), "hg_readback_end")
        while pending:
            got.append(ctx.readback_end(W, H))
            pending -= 1
        frames_of = [1, 2, 3, 4, 5, 6, 6]
        assert len(got) == len(frames_of)
        for img, f in zip(got, frames_of):
            host = abi.pack_display(want[f - 1], fmt)
            assert img.shape == host.shape and img.dtype == host.dtype
            bad = int((_bits(img) != _bits(host)).sum())
            assert bad == 0, f"format {fmt}, frame {f}: {bad} values differ from the host packing"
        assert_bitwise(ctx.readback(W, H), want[-1], "accumulation target after the display readbacks")


@pytest.mark.gpu
def test_gpu_display_format_tiling(gpu):
    """With a tiling, the other ranks' pixels pack as 0 in every format."""
    packed, params, cube, frames, acc = cases.setup("c1_64")
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    own, _ = gpu_render(packed, params, 2, True, cube, tiling=(1, 3))
    mine = ~np.isnan(own[..., 0])
    with abi.Context(0) as ctx:
        ctx.upload_scene(packed)
        ctx.resize(W, H)
        ctx.set_tiling(1, 3)
        ctx.set_params(params)
        ctx.render(2, True)
        for fmt in FORMATS:
            ctx.readback_begin(fmt)
            img = ctx.readback_end(W, H)
            host = abi.pack_display(np.where(mine[..., None], own, 0).astype(np.float32), fmt)
            assert int((_bits(img) != _bits(host)).sum()) == 0, fmt


@pytest.mark.gpu
def test_gpu_render_pass_display_latency_and_clear(gpu):
    """The Python HalogenRenderPass's display (as the C# and C++ passes): by default (latency 0, the reference's) each
    display() returns the frame just traced; with latency 1, the previous frame's image.  A camera move
    (ClearAccumulation, RP:262-268; the first frame's resolution setup is one too) ends the readbacks in flight unseen
    and shows the first frame after it at once, so no image from before the clear is ever shown."""
    from halogen import render_pass as rp, scenes
    from halogen.unity import Transform
    cfg = scenes.CONFIGS["C1"].resized(40, 32, 4)
    scene = cfg.build_scene()
    cam = cfg.camera()
    t = cam.transform
    moved = rp.Camera(Transform((t.position[0] + 0.05, t.position[1], t.position[2]), tuple(t.rotation)),
                      cam.fieldOfView, cam.pixelWidth, cam.pixelHeight)
    views = [cam] * 4 + [moved] * 3
    ref = rp.HalogenRenderPass(cfg.settings)
    want = []
    for c in views:
        ref.Execute(scene, c)
        want.append(abi.pack_display(ref.read_image(), abi.HG_DISPLAY_R11G11B10F))
    ref.Dispose()
    p = rp.HalogenRenderPass(cfg.settings)
    assert p.display_latency == 0
    for k in range(2):
        p.Execute(scene, views[k])
        assert np.array_equal(p.display(), want[k]), k
    p.Dispose()
    p = rp.HalogenRenderPass(cfg.settings)
    p.set_display(abi.HG_DISPLAY_R11G11B10F, 1)
    got = []
    for c in views:
        p.Execute(scene, c)
        got.append(p.display())
    # the first frame follows a clear too (the first OnCameraSetup's): shown at once, then the pipeline fills
    assert np.array_equal(got[0], want[0])
    assert got[1] is None
    for k in (2, 3):
        assert np.array_equal(got[k], want[k - 1]), k
    assert np.array_equal(got[4], want[4]), "the first frame after the camera move, shown at once"
    assert got[5] is None  # the pipeline refills behind it
    assert np.array_equal(got[6], want[5])
    assert np.array_equal(p.flush_display(), want[6])
    p.set_display(abi.HG_DISPLAY_RGBA16F, 0)  # at once
    p.Execute(scene, moved)
    img = p.display()
    assert img.dtype == np.float16 and np.array_equal(img.view(np.uint16),
                                                       abi.pack_display(p.read_image(), abi.HG_DISPLAY_RGBA16F).view(np.uint16))
    p.Dispose()
