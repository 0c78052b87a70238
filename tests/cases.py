"""Parity cases shared by tests/ and tools/make_goldens.py.  Each case = a scene, a camera/resolution, settings
overrides and a frame count; inputs are rebuilt deterministically from halogen.scenes."""
from __future__ import annotations

import hashlib
from dataclasses import replace
from functools import lru_cache

from halogen import render_pass as rp
from halogen import scenes

# name: (config, width, height, frames, accumulate, overrides)
CASES = {
    "c1_64": ("C1", 64, 64, 4, True, {}),
    "c1_256": ("C1", 256, 256, 1, True, {}),  # BASELINE.json configs[0]: the Cornell box at 256x256, 1 spp
    "c1_64_spp3": ("C1", 64, 64, 1, True, {"SamplesPerPixel": 3}),
    "c1_48_noacc": ("C1", 48, 48, 2, False, {"Accumulate": False}),
    "c1_40x24_bounce12": ("C1", 40, 24, 3, True, {"MaxBounces": 12, "DiffuseBounces": 12}),
    "c1_32_albedo": ("C1", 32, 32, 1, True, {"DebugMode": "Albedo"}),
    "c1_32_normal": ("C1", 32, 32, 1, True, {"DebugMode": "Normal"}),
    "c1_32_tritests": ("C1", 32, 32, 1, True, {"DebugMode": "RayTriangleTests", "FirstInteractionOnly": False}),
    "c1_32_boxtests": ("C1", 32, 32, 1, True, {"DebugMode": "RayBoxTests"}),
    "c1_32_combined": ("C1", 32, 32, 1, True, {"DebugMode": "Combined", "FirstInteractionOnly": False}),
    "c1_32_aperture": ("C1", 32, 32, 2, True, {"ApertureAngle": 2.0, "FocalPlaneDistance": 7.0, "FilterRadius": 1.5}),
    "glass_64x36": ("C5", 64, 36, 2, True, {}),
    "dragon1_64x36": ("C3", 64, 36, 2, True, {"_subdiv": 1}),
    # the full 871,200-triangle dragon (C3's scene), 32-level BLAS: streaming kernel, distributed leaf test
    "dragon10_64x36": ("C3", 64, 36, 16, True, {}),  # 16 frames: at 1 spp most Cornell paths end black
    "dragon10_96x54_normal": ("C3", 96, 54, 1, True, {"DebugMode": "Normal"}),  # every dragon hit's normal
    "dragon10_48x27_tritests": ("C3", 48, 27, 1, True, {"DebugMode": "RayTriangleTests", "FirstInteractionOnly": False}),
}


@lru_cache(maxsize=8)
def _scene(scene_kind: str, subdiv: int):
    if scene_kind == "dragon":
        sc = scenes.dragon_cornell(subdiv)
    else:
        sc = {"cornell": scenes.cornell_box, "glass": scenes.nested_glass}[scene_kind]()
    return sc.pack()


def setup(name: str, first_frame: int = 1):
    cfg_name, w, h, frames, accumulate, ov = CASES[name]
    cfg = scenes.CONFIGS[cfg_name].resized(w, h, frames)
    ov = dict(ov)
    subdiv = ov.pop("_subdiv", 10)
    settings = replace(scenes.settings_for(cfg), **ov)
    packed = _scene(cfg.scene, subdiv)
    s = rp.clamp_settings(settings)
    cube = settings.environmentCubemap if s["UseEnvironmentCubemap"] else None
    params = rp.make_params(s, cfg.camera(), first_frame, len(packed.spheres), len(packed.meshes), cube is not None)
    return packed, params, cube, frames, accumulate


def setup_host(name: str):
    """The same case as the host sees it: scene, HalogenSettings and Camera (the uniforms are derived by the pass)."""
    cfg_name, w, h, frames, accumulate, ov = CASES[name]
    cfg = scenes.CONFIGS[cfg_name].resized(w, h, frames)
    ov = dict(ov)
    subdiv = ov.pop("_subdiv", 10)
    settings = replace(scenes.settings_for(cfg), **ov)
    return _scene(cfg.scene, subdiv), settings, cfg.camera(), frames, accumulate


def packed_digest(packed) -> str:
    h = hashlib.sha256()
    for k, v in packed.as_numpy().items():
        h.update(k.encode())
        h.update(v.tobytes())
    return h.hexdigest()
