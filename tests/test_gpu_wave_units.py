"""Multi-tile streaming waves (HG_OPT_WAVE_UNITS, csrc/hg_mega.hip UnitItems): a wave of a streaming launch without
the queue traces k consecutive tiles of the cost order, its lanes taking the k tiles' (pixel, frame) items one after
another.  Which wave traces an item changes nothing, so every image and counter must equal the one-tile-per-wave
render, the goldens and the oracle, bit for bit."""
import json
from pathlib import Path

import numpy as np
import pytest

import cases
import hg_oracle
from halogen import abi, render_pass as rp, scenes
from test_gpu_parity import assert_bitwise

GOLD = Path(__file__).resolve().parent / "golden"


def render(packed, params, frames, acc, cube, units, splits=None):
    with abi.Context(0) as ctx:
        ctx.set_option(abi.HG_OPT_KERNEL, abi.HG_KERNEL_MEGA_STREAM)
        ctx.set_option(abi.HG_OPT_WAVE_UNITS, units)
        W, H = int(params.screenParameters.x), int(params.screenParameters.y)
        ctx.upload_scene(packed)
        if cube is not None:
            ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
        ctx.resize(W, H)
        ctx.set_params(params)
        for n in (splits or [frames]):
            ctx.render(n, acc)
        img = np.full((H, W, 4), np.nan, np.float32)
        ctx.readback(W, H, img)
        return img, ctx.counters()


@pytest.mark.gpu
def test_gpu_wave_units_option_range(gpu):
    with abi.Context(0) as ctx:
        for v in (0, 1, 2, 4):
            ctx.set_option(abi.HG_OPT_WAVE_UNITS, v)
        for v in (-1, 5):
            with pytest.raises(abi.HalogenError, match="wave units"):
                ctx.set_option(abi.HG_OPT_WAVE_UNITS, v)


@pytest.mark.gpu
@pytest.mark.parametrize("units", [2, 3, 4])
@pytest.mark.parametrize("name", sorted(cases.CASES))
def test_gpu_wave_units_match_golden(gpu, name, units):
    meta = json.loads((GOLD / f"{name}.json").read_text())
    packed, params, cube, frames, acc = cases.setup(name)
    img, cnt = render(packed, params, frames, acc, cube, units)
    assert_bitwise(img, np.load(GOLD / f"{name}.npz")["image"], f"{name} wave units {units}")
    for k, v in meta["counters"].items():
        assert cnt[k] == v, (k, cnt[k], v)


@pytest.mark.gpu
@pytest.mark.parametrize("units", [2, 4])
def test_gpu_wave_units_chunks_bit_exact(gpu, units):
    """Launch chunks of 1, 3 and 12 frames (1-frame ones run the queue form, the others multi-tile waves) equal one
    16-frame launch with one tile per wave."""
    packed, params, cube, frames, acc = cases.setup("c1_64")
    ref, rc = render(packed, params, 16, True, cube, 1)
    img, c = render(packed, params, 16, True, cube, units, splits=[1, 3, 12])
    assert_bitwise(img, ref, f"1+3+12 frames, wave units {units}")
    for k in ("rays", "tri_tests", "aabb_tests", "hits"):
        assert c[k] == rc[k], (k, c[k], rc[k])


@pytest.mark.gpu
@pytest.mark.parametrize("units", [2, 4])
@pytest.mark.parametrize("cfg_name,rows", [("C3", (536, 540)), ("C2", (760, 763))])
def test_gpu_wave_units_full_size_rows_match_oracle(gpu, cfg_name, rows, units):
    cfg = scenes.CONFIGS[cfg_name]
    settings = scenes.settings_for(cfg)
    s = rp.clamp_settings(settings)
    packed = cases._scene(cfg.scene, 10)
    cube = settings.environmentCubemap if s["UseEnvironmentCubemap"] else None
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), cube is not None)
    img, _ = render(packed, params, 2, True, cube, units)
    W = cfg.width
    y0, y1 = rows
    ref, _ = hg_oracle.render(packed, params, 2, True, cubemap=cube, pix_range=(y0 * W, y1 * W))
    assert_bitwise(img[y0:y1], ref[y0:y1], f"{cfg_name} rows {rows}, wave units {units}")
    assert np.all(img[..., 3] == 1.0) and np.isfinite(img).all()
