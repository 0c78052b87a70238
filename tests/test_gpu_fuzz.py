"""Seeded random scenes, cameras and settings: every kernel against the live CPU oracle, bit for bit.

The golden cases pin fixed configurations; this sweeps the input space the reference's pass accepts around them
(RP:169-231 clamps, HC:876-950 bounce loop, HC:582-665 nested dielectrics): a Cornell box with random extra spheres
and rotated cubes (and in a third of the cases the 8.7k-triangle dragon) of random materials (diffuse, metal, rough glass with priorities and absorption, emissive), a
jittered and turned camera, random bounce limits, samples per pixel, aperture, filter radius, accumulation on or off,
and the synthetic environment cube map on or off.  Each case renders a small image for a few frames and must equal
the oracle's image bit for bit with equal work counters.  Parity here is against our restatement of the reference
(oracle/hg_oracle.c), as for every image test."""
from dataclasses import replace

import numpy as np
import pytest

import hg_oracle
from halogen import render_pass as rp, scenes
from halogen.render_pass import Camera
from halogen.scene import HalogenMaterial, RayTracingMesh, RayTracingSphere
from halogen.unity import Transform, euler_to_quat, unity_cube

from test_gpu_parity import KERNELS, assert_bitwise, gpu_render

SEEDS = list(range(24))
W, H = 40, 24


def _material(rng: np.random.Generator) -> HalogenMaterial:
    col = tuple(float(v) for v in rng.uniform(0.05, 1.0, 3)) + (1.0,)
    kind = rng.integers(4)
    if kind == 0:  # diffuse
        return HalogenMaterial.default(col)
    if kind == 1:  # metal / glossy
        return HalogenMaterial(color=col, specularColor=col, metallic=float(rng.uniform(0.1, 1.0)),
                               roughness=float(rng.uniform(0.0, 0.6)))
    if kind == 2:  # dielectric (albedo alpha < property sample: transmission), nested priorities, absorption
        return HalogenMaterial(color=col[:3] + (float(rng.uniform(0.0, 0.3)),), subsurfaceColor=col,
                               indexOfRefraction=float(rng.uniform(1.1, 1.8)), roughness=float(rng.uniform(0.0, 0.3)),
                               absorption=float(rng.uniform(0.0, 1.5)), dielectricPriority=int(rng.integers(0, 3)))
    return HalogenMaterial(color=col, emissionColor=col, emissionIntensity=float(rng.uniform(0.5, 4.0)))


def _case(seed: int):
    rng = np.random.default_rng(1000 + seed)
    sc = scenes.cornell_box()
    root = Transform(scenes.CORNELL_ROOT)
    for i in range(int(rng.integers(1, 5))):
        pos = (float(rng.uniform(-1.8, 1.8)), float(rng.uniform(-2.0, 1.5)), float(rng.uniform(14.2, 17.0)))
        sc.add(RayTracingSphere(f"Fuzz sphere {i}", Transform(pos, parent=root), float(rng.uniform(0.15, 0.6)),
                                _material(rng)))
    v, n, t = unity_cube()
    for i in range(int(rng.integers(0, 4))):
        pos = (float(rng.uniform(-1.8, 1.8)), float(rng.uniform(-2.0, 1.5)), float(rng.uniform(14.2, 17.0)))
        q = euler_to_quat(*(float(a) for a in rng.uniform(-180, 180, 3)))
        s = tuple(float(a) for a in rng.uniform(0.2, 0.9, 3))
        sc.add(RayTracingMesh(f"Fuzz cube {i}", v, n, t, Transform(pos, q, s, root), _material(rng)))
    if rng.integers(3) == 0:  # the 8.7k-triangle dragon (a deep BLAS: the streaming kernel's resumable traversal)
        dv, dn, dt = scenes.dragon_mesh(1)
        q = euler_to_quat(0.0, float(rng.uniform(0, 360)), 0.0)
        pos = (float(rng.uniform(-1.0, 1.0)), -0.991, float(rng.uniform(15.0, 16.5)))
        sc.add(RayTracingMesh("Fuzz dragon", dv, dn, dt, Transform(pos, q, (1.2, 1.2, 1.2), root), _material(rng)))
    packed = sc.pack()
    base = scenes.settings_for(scenes.CONFIGS["C1"])
    sky = bool(rng.integers(2))
    accumulate = bool(rng.integers(4) > 0)
    settings = replace(base, MaxBounces=int(rng.integers(1, 13)), DiffuseBounces=int(rng.integers(1, 9)),
                       GlossyBounces=int(rng.integers(1, 9)), TransmissionBounces=int(rng.integers(1, 13)),
                       SamplesPerPixel=int(rng.integers(1, 3)), Accumulate=accumulate,
                       ApertureAngle=float(rng.choice([0.0, 0.0, rng.uniform(0.2, 3.0)])),
                       FocalPlaneDistance=float(rng.uniform(4.0, 12.0)), FilterRadius=float(rng.uniform(0.3, 2.0)),
                       useHDRISky=sky, environmentCubemap=scenes.synthetic_sky() if sky else None,
                       EnvironmentMipLevel=int(rng.integers(0, 4)))
    s = rp.clamp_settings(settings)
    cube = settings.environmentCubemap if s["UseEnvironmentCubemap"] else None
    cam_pos = tuple(float(p + d) for p, d in zip(scenes.CORNELL_CAMERA_POS, rng.uniform(-0.6, 0.6, 3)))
    cam_rot = euler_to_quat(float(rng.uniform(-6, 6)), float(rng.uniform(-8, 8)), 0.0)
    camera = Camera(Transform(cam_pos, cam_rot), float(rng.uniform(40, 75)), W, H)
    params = rp.make_params(s, camera, 1, len(packed.spheres), len(packed.meshes), cube is not None)
    frames = int(rng.integers(1, 4))
    return packed, params, frames, accumulate, cube


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", sorted(KERNELS))
@pytest.mark.parametrize("seed", SEEDS)
def test_gpu_fuzz_matches_oracle(gpu, seed, kernel):
    packed, params, frames, acc, cube = _case(seed)
    img, cnt = gpu_render(packed, params, frames, acc, cube=cube, kernel=kernel)
    ref, rcnt = hg_oracle.render(packed, params, frames, acc, cubemap=cube)
    assert_bitwise(img, ref, f"fuzz seed {seed}, kernel {kernel}")
    for k in ("rays", "tri_tests", "aabb_tests", "hits"):
        assert cnt[k] == rcnt[k], (k, cnt[k], rcnt[k])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS[:12])
def test_gpu_fuzz_sah_tree_matches_oracle(gpu, seed):
    """The same random scenes with every mesh's hierarchy from hg_build_blas_sah (not the reference builder's):
    the kernel traverses any tree the reference's way, so it still equals the oracle on the same tree, bit for bit."""
    from halogen import scene as sc

    prev = sc.set_blas_builder("sah")
    try:
        packed, params, frames, acc, cube = _case(seed)
    finally:
        sc.set_blas_builder(prev)
    img, cnt = gpu_render(packed, params, frames, acc, cube=cube)
    ref, rcnt = hg_oracle.render(packed, params, frames, acc, cubemap=cube)
    assert_bitwise(img, ref, f"fuzz seed {seed} on SAH trees")
    for k in ("rays", "tri_tests", "aabb_tests", "hits"):
        assert cnt[k] == rcnt[k], (k, cnt[k], rcnt[k])
