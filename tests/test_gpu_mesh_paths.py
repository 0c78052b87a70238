"""GPU parity for the mesh-record paths the benchmark scenes never take.

The kernels copy every mesh's world->local matrix and header into the wave's LDS only while the table fits the
per-wave LDS budget (hg_mega.hip mesh_lds_bytes: 16 meshes for the streaming kernel, fewer for the regenerating
one); larger scenes read the records from global memory.  The exact mesh cull keeps a 64-bit live mask, so meshes
64 and beyond are never culled (hg_device.h mesh_live_mask).  The benchmark scenes have 7-10 meshes, so both paths
are exercised here: the Cornell box with a grid of extra cubes (30 and 75 meshes in all), every kernel, against the
live CPU oracle, bit for bit and with equal work counters."""
import numpy as np
import pytest

import hg_oracle
from halogen import render_pass as rp, scenes
from halogen.scene import HalogenMaterial, RayTracingMesh
from halogen.unity import Transform, unity_cube

from test_gpu_parity import KERNELS, assert_bitwise, gpu_render


def _cubes_scene(n_extra: int):
    """The C1 Cornell box plus n_extra small cubes on a grid inside it (distinct materials every 3rd cube)."""
    sc = scenes.cornell_box()
    root = Transform(scenes.CORNELL_ROOT)
    v, n, t = unity_cube()
    mats = [HalogenMaterial.default((0.9, 0.9, 0.9, 1.0)), HalogenMaterial.default((0.3, 0.6, 0.9, 1.0)),
            HalogenMaterial(color=(1, 1, 1, 1), metallic=0.7, roughness=0.2)]
    side = int(np.ceil(np.sqrt(n_extra)))
    for i in range(n_extra):
        gx, gy = i % side, i // side
        pos = (-2.0 + 4.0 * (gx + 0.5) / side, -2.0 + 3.5 * (gy + 0.5) / side, 17.6)
        q = (0.0, float(np.sin(0.1 * i)), 0.0, float(np.cos(0.1 * i)))
        sc.add(RayTracingMesh(f"Grid cube {i}", v, n, t, Transform(pos, q, (0.25, 0.25, 0.25), root), mats[i % 3]))
    return sc.pack()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", sorted(KERNELS))
@pytest.mark.parametrize("n_extra", [21, 66])
def test_gpu_many_meshes_match_oracle(gpu, n_extra, kernel):
    packed = _cubes_scene(n_extra)
    assert len(packed.meshes) == 9 + n_extra
    cfg = scenes.CONFIGS["C1"]
    settings = scenes.settings_for(cfg)
    s = rp.clamp_settings(settings)
    W, H, frames = 48, 32, 3
    params = rp.make_params(s, scenes.cornell_camera(W, H), 1, len(packed.spheres), len(packed.meshes), False)
    img, cnt = gpu_render(packed, params, frames, True, kernel=kernel)
    ref, rcnt = hg_oracle.render(packed, params, frames, True)
    assert_bitwise(img, ref, f"{len(packed.meshes)} meshes, kernel {kernel}")
    for k in ("rays", "tri_tests", "aabb_tests", "hits"):
        assert cnt[k] == rcnt[k], (k, cnt[k], rcnt[k])
    assert rcnt["hits"] > 0.3 * rcnt["paths"], "the grid is not in view: not a parity check"
