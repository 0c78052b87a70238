"""Files the native host (halogen-pathtracer_amd/host/halogen_render, the C++ HalogenRenderPass) reads: the packed
scene buffers, the cubemap, and the settings + camera as "key value" lines (formats in halogen_render.cpp)."""
from __future__ import annotations

import struct
from pathlib import Path

import numpy as np

from . import render_pass as rp
from .unity import to_unity_floats

SETTING_KEYS = ("ShowInSceneView", "Accumulate", "SamplesPerPixel", "MaxAccumulatedFrames", "UnlimitedSampling",
                "MaxBounces", "DiffuseBounces", "GlossyBounces", "TransmissionBounces", "FilterRadius",
                "NearPlaneDistance", "FarPlaneDistance", "FocalPlaneDistance", "ApertureAngle", "useHDRISky",
                "EnvironmentMipLevel", "FirstInteractionOnly", "TriangleDebugDisplayRange", "BoxDebugDisplayRange")


def write_scene(packed, path) -> None:
    """HGSCENE1: counts, then the reference-layout arrays as hg_upload_scene takes them."""
    arrays = (packed.spheres, packed.meshes, packed.materials, packed.triangles, packed.blas)
    with open(path, "wb") as f:
        f.write(b"HGSCENE1")
        f.write(struct.pack("<5i", *(len(a) for a in arrays)))
        for a in arrays:
            f.write(bytes(a))


def write_cubemap(cube, path) -> None:
    t = np.ascontiguousarray(cube.texels, dtype=np.float32)
    with open(path, "wb") as f:
        f.write(b"HGCUBE01")
        f.write(struct.pack("<iiq", cube.face_size, cube.n_mips, t.size))
        f.write(t.tobytes())


def _v(x) -> str:
    if isinstance(x, bool):
        return "1" if x else "0"
    if isinstance(x, (int, np.integer)):
        return str(int(x))
    return repr(float(x))


def write_config(settings: rp.HalogenSettings, camera: rp.Camera, path, frames: int = 1, frame_count: int = 1,
                 n_spheres: int = 0, n_meshes: int = 0, cubemap_path: str | None = None) -> None:
    lines = [f"width {camera.pixelWidth}", f"height {camera.pixelHeight}", f"fov {_v(camera.fieldOfView)}",
             "position " + " ".join(_v(v) for v in camera.transform.position),
             "rotation " + " ".join(_v(v) for v in camera.transform.rotation),
             "localToWorld " + " ".join(_v(v) for v in to_unity_floats(camera.transform.local_to_world)),
             f"frames {frames}", f"frame_count {frame_count}", f"n_spheres {n_spheres}", f"n_meshes {n_meshes}"]
    for k in SETTING_KEYS:
        lines.append(f"{k} {_v(getattr(settings, k))}")
    mode = settings.DebugMode
    lines.append(f"DebugMode {rp.DEBUG_MODES.get(mode, 0) if isinstance(mode, str) else int(mode)}")
    if cubemap_path:
        lines.append(f"cubemap {cubemap_path}")
    Path(path).write_text("\n".join(lines) + "\n")
