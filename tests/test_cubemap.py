"""Seamless cube-map filtering (TextureCube.SampleLevel, HC:201; the reference's cubemap is imported
seamlessCubemap: 1, resting_place_4k.exr.meta:32, and D3D10+ filters every cube seamlessly).

CPU: the oracle's integer face adjacency equals an independent float re-projection of the extended face plane, is
symmetric, and makes sampling continuous across face edges (where a per-face clamp jumps).  GPU: an empty scene
(every camera ray misses, pixel = sky(dir, DefaultMip)) looked at along a cube corner shows three faces, their edges
and the corner at four mip levels; the kernel's image equals the oracle's bit for bit."""
import dataclasses

import numpy as np
import pytest

import hg_oracle
from halogen import envmap, render_pass as rp
from halogen.scene import Scene
from halogen.unity import Transform, euler_to_quat

M = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], float)
S = np.array([[0, 0, -1], [0, 0, 1], [1, 0, 0], [1, 0, 0], [1, 0, 0], [-1, 0, 0]], float)
T = np.array([[0, -1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1], [0, -1, 0], [0, -1, 0]], float)


def reproject(f, i, j, size):
    """The texel of the cube face the direction through texel (i, j)'s centre on face f's extended plane lands in."""
    sc, tc = 2 * (i + 0.5) / size - 1, 2 * (j + 0.5) / size - 1
    d = M[f] + sc * S[f] + tc * T[f]
    k = int(np.argmax(np.abs(d)))
    g = 2 * k + (1 if d[k] < 0 else 0)
    ma = abs(d[k])
    s2, t2 = (d @ S[g] / ma + 1) / 2, (d @ T[g] / ma + 1) / 2
    return g, min(size - 1, int(np.floor(s2 * size))), min(size - 1, int(np.floor(t2 * size)))


def off_face_texels(size):
    for f in range(6):
        for k in range(size):
            for i, j in ((-1, k), (size, k), (k, -1), (k, size)):
                yield f, i, j


@pytest.mark.parametrize("size", [1, 2, 3, 4, 7, 16])
def test_adjacency_equals_reprojection_and_is_symmetric(built, size):
    for f, i, j in off_face_texels(size):
        g, ii, jj = hg_oracle.cube_adjacent(f, i, j, size)
        assert (g, ii, jj) == reproject(f, i, j, size), (f, i, j)
        assert g != f and 0 <= ii < size and 0 <= jj < size
        # stepping back off face g across the same edge returns to the original face's edge texel
        back = [(g, ii + di, jj + dj) for di, dj in ((-1, 0), (1, 0), (0, -1), (0, 1))
                if not (0 <= ii + di < size and 0 <= jj + dj < size)]
        origin = (f, min(max(i, 0), size - 1), min(max(j, 0), size - 1))
        assert any(hg_oracle.cube_adjacent(*b, size) == origin for b in back), (f, i, j)


def _random_cube(size, mips, seed=1):
    rng = np.random.default_rng(seed)
    n = sum(6 * max(1, size >> m) ** 2 * 4 for m in range(mips))
    return envmap.Cubemap(size, mips, rng.random(n, dtype=np.float32) * 4.0)


def test_sampling_is_continuous_across_face_edges(built):
    cube = _random_cube(8, 2)
    rng = np.random.default_rng(7)
    for _ in range(200):
        # a point on an edge of the cube [-1,1]^3: two coordinates at +-1, one free
        p = rng.choice([-1.0, 1.0], 3)
        p[rng.integers(3)] = rng.uniform(-0.95, 0.95)
        free = np.argmax(np.abs(p) < 1)
        e = np.zeros(3)
        for k in range(3):
            if k != free:
                e[k] = p[k]
        # step off the edge into each of the two faces
        fixed = [k for k in range(3) if k != free]
        eps = 2e-4
        a = p.copy()
        a[fixed[1]] *= 1 - eps  # face of axis fixed[0]
        b = p.copy()
        b[fixed[0]] *= 1 - eps  # face of axis fixed[1]
        for level in (0, 1):
            va, vb = hg_oracle.cube_sample(cube, a, level), hg_oracle.cube_sample(cube, b, level)
            assert np.allclose(va, vb, atol=0.05), (p, level, va, vb)


def _sky_case(w, h, mip, cube):
    settings = dataclasses.replace(rp.HalogenSettings(), useHDRISky=True, environmentCubemap=cube,
                                   EnvironmentMipLevel=mip)
    s = rp.clamp_settings(settings)
    cam = rp.Camera(Transform((0, 0, 0), euler_to_quat(-35.26439, 45.0, 0.0)), 100.0, w, h)
    packed = Scene().pack()
    params = rp.make_params(s, cam, 1, 0, 0, True)
    return packed, params


@pytest.mark.gpu
@pytest.mark.parametrize("mip", [0, 1, 3, 5])
def test_gpu_sky_corner_matches_oracle(gpu, mip):
    from halogen import abi
    from test_gpu_parity import assert_bitwise

    cube = _random_cube(32, 6)
    packed, params = _sky_case(96, 64, mip, cube)
    ref, _ = hg_oracle.render(packed, params, 1, True, cubemap=cube)
    with abi.Context(0) as ctx:
        ctx.upload_scene(packed)
        ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
        ctx.resize(96, 64)
        ctx.set_params(params)
        ctx.render(1, True)
        img = ctx.readback(96, 64)
    assert (ref[..., :3] > 0).all()
    assert_bitwise(img, ref, f"sky at mip {mip}")
