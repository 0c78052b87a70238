"""hg_upload_scene re-uploads (VERDICT r03 missing #3).  The reference re-runs UpdateObjectBuffers + SetBufferData on
every camera move (ClearAccumulation sets ObjectBuffersDirty, HalogenRenderPass.cs:262-268, 296-299, 448-509), and the
drop-in keeps that call pattern, so the library detects an upload of the arrays it already holds (byte equality against
retained host copies) and changes nothing.  These tests check that a skipped upload really is a no-op (the image stays
bit-identical to an uninterrupted render, with the tile cost order carried on), that equality is by content (fresh
copies of the arrays are skipped too), and that any changed byte rebuilds the device scene."""
import ctypes as C

import numpy as np
import pytest

import cases
from halogen import abi
from halogen.scene import PackedScene
from test_gpu_parity import assert_bitwise, gpu_render


def _copy(packed):
    arrays = {}
    for k in ("spheres", "meshes", "materials", "triangles", "blas"):
        a = getattr(packed, k)
        b = (type(a)._type_ * len(a))()
        C.memmove(b, a, C.sizeof(a))
        arrays[k] = b
    return PackedScene(**arrays)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["dragon10_64x36", "glass_64x36"])
def test_gpu_identical_reupload_is_a_noop(gpu, name):
    packed, params, cube, frames, acc = cases.setup(name)
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    want, wcnt = gpu_render(packed, params, 6, True, cube)
    with abi.Context(0) as ctx:
        ctx.upload_scene(packed)
        if cube is not None:
            ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
        ctx.resize(W, H)
        ctx.set_params(params)
        ctx.render(2, True)
        ctx.upload_scene(packed)        # the same arrays
        ctx.render(2, True)
        ctx.upload_scene(_copy(packed))  # equal content in other buffers
        ctx.render(2, True)
        img = ctx.readback(W, H)
        cnt = ctx.counters()
    assert cnt["scene_uploads"] == 1 and cnt["scene_uploads_skipped"] == 2, cnt
    assert_bitwise(img, want, f"{name}: 2 + 2 + 2 frames around two identical re-uploads")
    for k in ("paths", "rays", "tri_tests", "aabb_tests"):
        assert cnt[k] == wcnt[k], k


@pytest.mark.gpu
def test_gpu_changed_reupload_rebuilds(gpu):
    packed, params, cube, frames, acc = cases.setup("c1_64")
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    changed = _copy(packed)
    changed.materials[0].albedo.x = np.float32(changed.materials[0].albedo.x) * np.float32(0.5)
    moved = _copy(packed)
    moved.triangles[len(moved.triangles) - 1].pointA.x += 1e-3  # one float of one triangle
    for variant in (changed, moved):
        want, _ = gpu_render(variant, params, 3, True)
        with abi.Context(0) as ctx:
            ctx.upload_scene(packed)
            ctx.resize(W, H)
            ctx.set_params(params)
            ctx.render(1, True)
            ctx.upload_scene(variant)
            ctx.clear_accumulation()
            ctx.set_params(params)
            ctx.render(3, True)
            img = ctx.readback(W, H)
            cnt = ctx.counters()
        assert cnt["scene_uploads"] == 2 and cnt["scene_uploads_skipped"] == 0, cnt
        assert_bitwise(img, want, "after a changed re-upload")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["dragon1_64x36", "glass_64x36"])
def test_gpu_partial_reupload_equals_full(gpu, name):
    """An object moved (one mesh's world->local matrix), a material and a sphere changed, the triangles and BVH entries
    as before: only the mesh table, spheres and materials are rebuilt (hg_counters.scene_uploads_partial), and the
    render equals a fresh context's full upload of the same arrays, bit for bit."""
    packed, params, cube, frames, acc = cases.setup(name)
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    moved = _copy(packed)
    moved.meshes[0].worldToLocal.m[12] += np.float32(0.05)  # translate the first mesh
    moved.materials[0].roughness = np.float32(0.25)
    if len(moved.spheres):
        moved.spheres[0].radius = np.float32(moved.spheres[0].radius * 0.9)
    want, wcnt = gpu_render(moved, params, 3, True, cube)
    with abi.Context(0) as ctx:
        ctx.upload_scene(packed)
        if cube is not None:
            ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
        ctx.resize(W, H)
        ctx.set_params(params)
        ctx.render(2, True)
        ctx.upload_scene(moved)
        ctx.clear_accumulation()
        ctx.set_params(params)
        ctx.render(3, True)
        img = ctx.readback(W, H)
        cnt = ctx.counters()
    assert cnt["scene_uploads"] == 2 and cnt["scene_uploads_partial"] == 1 and cnt["scene_uploads_skipped"] == 0, cnt
    assert_bitwise(img, want, f"{name}: partial re-upload vs a fresh full upload")
