"""GPU parity for both forms of the camera ray (hg_device.h camera_ray).

With a focal-disc radius of 0 the kernels skip the focal-disc sample and its sincos (HG_PINHOLE_FAST): the aperture
point is (+-0, +-0, 0) and its zeros cannot reach the ray as long as no camera translation component is 0.  The
benchmark cameras take that form.  A camera with a zero translation component takes the full form even at aperture 0,
and so does any aperture (the c1_32_aperture golden).  Both are checked here against the live CPU oracle, bit for bit
and with equal work counters, on every kernel."""
import pytest

import hg_oracle
from halogen import render_pass as rp, scenes
from halogen.render_pass import Camera
from halogen.unity import Transform

from test_gpu_parity import KERNELS, assert_bitwise, gpu_render

W, H, FRAMES = 48, 32, 2
CAMERAS = {
    "pinhole_fast": scenes.CORNELL_CAMERA_POS,                          # every component nonzero: the short form
    "pinhole_x0": (0.0,) + tuple(scenes.CORNELL_CAMERA_POS[1:]),         # translation x == 0: the full form
    "pinhole_y_neg0": (scenes.CORNELL_CAMERA_POS[0], -0.0, scenes.CORNELL_CAMERA_POS[2]),  # -0: the full form too
}


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", sorted(KERNELS))
@pytest.mark.parametrize("cam", sorted(CAMERAS))
def test_gpu_camera_forms_match_oracle(gpu, cam, kernel):
    packed = scenes.cornell_box().pack()
    cfg = scenes.CONFIGS["C1"]
    s = rp.clamp_settings(scenes.settings_for(cfg))
    camera = Camera(Transform(CAMERAS[cam], (0, 0, 0, 1)), 60.0, W, H)
    params = rp.make_params(s, camera, 1, len(packed.spheres), len(packed.meshes), False)
    # the translation's zero components (the form the kernel takes) are those of the position
    assert [v == 0.0 for v in params.camLocalToWorld.m[12:15]] == [c == 0.0 for c in CAMERAS[cam]]
    img, cnt = gpu_render(packed, params, FRAMES, True, kernel=kernel)
    ref, rcnt = hg_oracle.render(packed, params, FRAMES, True)
    assert_bitwise(img, ref, f"camera {cam}, kernel {kernel}")
    for k in ("rays", "tri_tests", "aabb_tests", "hits"):
        assert cnt[k] == rcnt[k], (k, cnt[k], rcnt[k])
    assert rcnt["hits"] > 0.3 * rcnt["paths"], "the box is not in view: not a parity check"
