"""The benchmark / parity scenes C1..C5 and their settings.

Scene constants come from Assets/Scenes/Testing Scene.unity (Cornell Box root :2353-2378, walls, light
cube with emission 5 at :1588, interior cubes) and the renderer asset (Assets/URP-HighFidelity-Renderer.asset:51-77).
The 871k-triangle dragon does not exist in the reference (Dragon_87k.fbx is a missing blob,
.MISSING_LARGE_BLOBS:1-3), so it is Dragon_8k.fbx (assets/dragon_8k.npz, tools/convert_dragon.py)
uniformly subdivided 10x per edge: 8,712 x 100 = 871,200 triangles.  The camera of the Cornell screenshot
is not stored in the scene, so CORNELL_CAMERA defines one (centred on the open front, looking +Z).
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from pathlib import Path

import numpy as np

from .envmap import Cubemap, synthetic_sky
from .render_pass import Camera, HalogenSettings
from .scene import HalogenMaterial, RayTracingMesh, RayTracingSphere, Scene
from .unity import Transform, euler_to_quat, unity_cube, unity_plane

ASSETS = Path(__file__).resolve().parents[2] / "assets"

# Constants of the "Cornell Box" subtree of Testing Scene.unity, exactly as the file writes them (float32 shortest
# round-trip decimals, -0 kept), pinned by tests/test_scene_constants.py against tests/golden/unity_scene.json
# (tools/extract_unity_scene.py parses the reference files into that fixture).
CORNELL_ROOT = (3.48, 1.24, 1.55)  # Testing Scene.unity:2378 (rotation identity, scale 1)

WHITE = HalogenMaterial.default((1.0, 1.0, 1.0, 1.0))
CYAN = HalogenMaterial(color=(0.0, 0.8414836, 1.0, 1.0))         # Plane (2), :544
RED = HalogenMaterial(color=(1.0, 0.27699995, 0.27699995, 1.0))  # Plane (3), :874
LIGHT = HalogenMaterial(color=(1, 1, 1, 1), specularColor=(1, 1, 1, 1), subsurfaceColor=(1, 1, 1, 1),
                        emissionColor=(1, 1, 1, 1), emissionIntensity=5.0)  # Light, :1566-1588
CUBE1 = HalogenMaterial(color=(1, 1, 1, 1), specularColor=(1, 1, 1, 1),
                        subsurfaceColor=(1.0, 0.13679248, 0.13679248, 1.0), indexOfRefraction=1.1)  # Cube (1), :9333
DRAGON = HalogenMaterial(color=(0.4716981, 0.4716981, 0.4716981, 1.0), metallic=0.5)  # Dragon_87k instance, :814-823
DIFFUSE_SPHERE = HalogenMaterial.default((0.2, 0.75, 0.3, 1.0))
GLASS_SPHERE = HalogenMaterial(color=(1.0, 1.0, 1.0, 0.05), roughness=0.05, metallic=0.02,
                               subsurfaceColor=(1.0, 0.55, 0.55, 1.0), indexOfRefraction=1.5, absorption=0.3)

# (name, built-in mesh, local position, local rotation (x, y, z, w), local scale, material); children of the root
CORNELL_WALLS = [
    ("Plane", "Plane", (0, -2.5, 16), (0, 0, 0, 1), (0.5, 1, 0.5), WHITE),
    ("Plane (4)", "Plane", (0, 2.5, 16), (0, 0, 1, 0), (0.5, 1, 0.5), WHITE),
    ("Plane (1)", "Plane", (0, 0, 18.5), (-0.7071068, 0, 0, 0.7071068), (0.5, 1, 0.5), WHITE),
    ("Plane (2)", "Plane", (2.5, 0, 16), (-0.5, 0.5, 0.5, 0.5), (0.5, 1, 0.5), CYAN),
    ("Plane (3)", "Plane", (-2.5, 0, 16), (-0.5, -0.5, -0.5, 0.5), (0.5, 1, 0.5), RED),
]
CORNELL_LIGHT = ("Light", "Cube", (0, 2.47, 16.24), (0, 0, 0, 1), (1.5, 0.25, 1.5), LIGHT)
CORNELL_FRONT_PANEL_ACTIVE = False  # "Front Panel" (z 13.5) is inactive in the scene: the box is open
# children of "Basic Interior" (identity transform under the root)
CORNELL_INTERIOR = [
    ("Cube", "Cube", (-1.1599998, -1.25, 16.83), (-0.0, -0.14046915, -0.0, 0.99008507), (1.4999999, 2.5, 1.4999999),
     WHITE),
    ("Cube (1)", "Cube", (0.91, -1.53, 15.85), (-0.0, 0.2588186, -0.0, 0.965926), (1.5, 1.5, 1.5), CUBE1),
    ("Cube (3)", "Cube", (-0.7750001, -2.37, 14.860999), (-0.0, 0.115712814, -0.0, 0.99328274), (1.2, 0.25, 1.2),
     WHITE),
]


def _cornell_shell(scene: Scene, root: Transform, with_interior: bool):
    meshes = {"Plane": unity_plane(), "Cube": unity_cube()}
    objects = CORNELL_WALLS + [CORNELL_LIGHT] + (CORNELL_INTERIOR if with_interior else [])
    for name, mesh, pos, q, scale, mat in objects:
        v, n, t = meshes[mesh]
        scene.add(RayTracingMesh(name, v, n, t, Transform(pos, q, scale, root), mat))


def cornell_box() -> Scene:
    """C1/C2: the reference Cornell box (5 walls, light cube, 3 interior cubes) + 2 spheres."""
    scene = Scene()
    root = Transform(CORNELL_ROOT)
    _cornell_shell(scene, root, with_interior=True)
    scene.add(RayTracingSphere("Diffuse Sphere", Transform((0.91, -0.28, 15.85), parent=root), 0.5, DIFFUSE_SPHERE))
    scene.add(RayTracingSphere("Glass Sphere", Transform((-0.775, -1.745, 14.861), parent=root), 0.5, GLASS_SPHERE))
    return scene


def subdivide(verts: np.ndarray, norms: np.ndarray, tris: np.ndarray, n: int):
    """Uniform n x n subdivision of every triangle (n^2 children).  Points are computed in float64 from
    barycentric coordinates and rounded to float32; normals are interpolated and renormalised."""
    if n <= 1:
        return verts, norms, tris
    ij = [(i, j) for i in range(n + 1) for j in range(n + 1 - i)]
    lut = {p: k for k, p in enumerate(ij)}
    bu = np.array([i / n for i, _ in ij])[None, :, None]
    bv = np.array([j / n for _, j in ij])[None, :, None]
    A = verts[tris[:, 0]].astype(np.float64)[:, None, :]
    B = verts[tris[:, 1]].astype(np.float64)[:, None, :]
    Cc = verts[tris[:, 2]].astype(np.float64)[:, None, :]
    P = A * (1.0 - bu - bv) + B * bu + Cc * bv
    nA = norms[tris[:, 0]].astype(np.float64)[:, None, :]
    nB = norms[tris[:, 1]].astype(np.float64)[:, None, :]
    nC = norms[tris[:, 2]].astype(np.float64)[:, None, :]
    N = nA * (1.0 - bu - bv) + nB * bu + nC * bv
    N /= np.linalg.norm(N, axis=2, keepdims=True)
    local = []
    for i in range(n):
        for j in range(n - i):
            local.append((lut[(i, j)], lut[(i + 1, j)], lut[(i, j + 1)]))
            if i + j < n - 1:
                local.append((lut[(i + 1, j)], lut[(i + 1, j + 1)], lut[(i, j + 1)]))
    local = np.array(local, dtype=np.int64)
    k = len(ij)
    base = (np.arange(len(tris), dtype=np.int64) * k)[:, None, None]
    out_t = (base + local[None, :, :]).reshape(-1, 3).astype(np.int32)
    return P.reshape(-1, 3).astype(np.float32), N.reshape(-1, 3).astype(np.float32), out_t


def dragon_mesh(subdiv: int = 10):
    d = np.load(ASSETS / "dragon_8k.npz", allow_pickle=False)
    return subdivide(d["vertices"], d["normals"], d["triangles"], subdiv)


def dragon_cornell(subdiv: int = 10) -> Scene:
    """C3/C4: Cornell walls + light + the 871,200-triangle dragon + the 2 spheres."""
    scene = Scene()
    root = Transform(CORNELL_ROOT)
    _cornell_shell(scene, root, with_interior=False)
    v, n, t = dragon_mesh(subdiv)
    scene.add(RayTracingMesh(f"Dragon x{subdiv}", v, n, t,
                             Transform((0.0, -0.991, 16.0), euler_to_quat(0, 90, 0), (1.6, 1.6, 1.6), root), DRAGON))
    scene.add(RayTracingSphere("Diffuse Sphere", Transform((-1.6, -2.0, 14.8), parent=root), 0.5, DIFFUSE_SPHERE))
    scene.add(RayTracingSphere("Glass Sphere", Transform((1.6, -2.0, 14.8), parent=root), 0.5, GLASS_SPHERE))
    return scene


def nested_glass() -> Scene:
    """C5: a glass sphere nested inside a glass cube (priorities 0 inside 1), absorbing, on a floor,
    lit by the synthetic environment cubemap."""
    scene = Scene()
    pv, pn, pt = unity_plane()
    cv, cn, ct = unity_cube()
    cube_glass = HalogenMaterial(color=(1.0, 1.0, 1.0, 0.1), roughness=0.04, metallic=0.02,
                                 subsurfaceColor=(0.6, 0.85, 1.0, 1.0), indexOfRefraction=1.5, absorption=0.25,
                                 dielectricPriority=1)
    sphere_glass = HalogenMaterial(color=(1.0, 1.0, 1.0, 0.1), roughness=0.0, metallic=0.02,
                                   subsurfaceColor=(1.0, 0.45, 0.3, 1.0), indexOfRefraction=1.33, absorption=0.8,
                                   dielectricPriority=0)
    floor = HalogenMaterial.default((0.6, 0.6, 0.6, 1.0))
    scene.add(RayTracingMesh("Floor", pv, pn, pt, Transform((0, 0, 0), (0, 0, 0, 1), (2.0, 1.0, 2.0)), floor))
    scene.add(RayTracingMesh("Glass Cube", cv, cn, ct,
                             Transform((0.0, 1.01, 0.0), euler_to_quat(0, 30, 0), (2.0, 2.0, 2.0)), cube_glass))
    scene.add(RayTracingSphere("Inner Sphere", Transform((0.0, 1.01, 0.0)), 0.6, sphere_glass))
    scene.add(RayTracingSphere("Side Sphere", Transform((-2.2, 0.7, 1.0)), 0.7, GLASS_SPHERE))
    return scene


CORNELL_CAMERA_POS = (CORNELL_ROOT[0], CORNELL_ROOT[1], CORNELL_ROOT[2] + 8.7)
# The same camera moved in until the 5 x 5 opening of the box (local z 13.5) fills a 16:9 frame: at a 60 degree
# vertical FOV the frame is 2 d tan(30) * 16/9 = 2.053 d wide at distance d, so d = 5 / 2.053 = 2.436 puts the
# opening's side edges at the frame's edges and every camera ray enters the box (bench.py "framed" measurement).
CORNELL_FRAMED_CAMERA_POS = (CORNELL_ROOT[0], CORNELL_ROOT[1], CORNELL_ROOT[2] + 13.5 - 2.436)
GLASS_CAMERA_POS = (0.0, 2.2, -6.5)


def cornell_camera(w: int, h: int) -> Camera:
    return Camera(Transform(CORNELL_CAMERA_POS, (0, 0, 0, 1)), 60.0, w, h)


def cornell_framed_camera(w: int, h: int) -> Camera:
    return Camera(Transform(CORNELL_FRAMED_CAMERA_POS, (0, 0, 0, 1)), 60.0, w, h)


def glass_camera(w: int, h: int) -> Camera:
    return Camera(Transform(GLASS_CAMERA_POS, euler_to_quat(10, 0, 0)), 60.0, w, h)


@dataclass(frozen=True)
class Config:
    name: str
    scene: str          # "cornell" | "dragon" | "glass"
    width: int
    height: int
    frames: int
    settings: HalogenSettings
    gpus: int = 1
    view: str = "front"  # "front": CORNELL_CAMERA; "framed": the box opening fills the frame

    def build_scene(self) -> Scene:
        return {"cornell": cornell_box, "dragon": dragon_cornell, "glass": nested_glass}[self.scene]()

    def camera(self) -> Camera:
        if self.scene == "glass":
            return glass_camera(self.width, self.height)
        return (cornell_framed_camera if self.view == "framed" else cornell_camera)(self.width, self.height)

    def resized(self, w: int, h: int, frames: int | None = None) -> "Config":
        return replace(self, width=w, height=h, frames=self.frames if frames is None else frames)


_BASE = HalogenSettings(useHDRISky=False)  # the Cornell configs have no cubemap
CONFIGS = {
    "C1": Config("C1 cornell 256x256 1spp", "cornell", 256, 256, 1, _BASE),
    "C2": Config("C2 cornell 1080p 256spp 8 diffuse bounces", "cornell", 1920, 1080, 256,
                 replace(_BASE, MaxBounces=8, DiffuseBounces=8)),
    "C3": Config("C3 dragon-871k cornell 1080p 64spp 8 bounces", "dragon", 1920, 1080, 64,
                 replace(_BASE, MaxBounces=8, DiffuseBounces=8, GlossyBounces=8)),
    # C3 seen from inside the opening (no primary misses): the cost of a traced path without the open-front share
    "C3F": Config("C3 dragon-871k cornell 1080p 64spp 8 bounces, box opening filling the frame", "dragon", 1920, 1080,
                  64, replace(_BASE, MaxBounces=8, DiffuseBounces=8, GlossyBounces=8), view="framed"),
    "C4": Config("C4 dragon-871k cornell 4K 256spp 8 bounces 8 GPUs", "dragon", 3840, 2160, 256,
                 replace(_BASE, MaxBounces=8, DiffuseBounces=8, GlossyBounces=8), gpus=8),
    "C5": Config("C5 nested glass + env cubemap 1080p 64spp 12 transmission bounces", "glass", 1920, 1080, 64,
                 HalogenSettings(useHDRISky=True, environmentCubemap="synthetic", MaxBounces=16, DiffuseBounces=4,
                                 GlossyBounces=4, TransmissionBounces=12)),
}


def settings_for(cfg: Config) -> HalogenSettings:
    """Resolve the synthetic cubemap placeholder."""
    if cfg.settings.environmentCubemap == "synthetic":
        return replace(cfg.settings, environmentCubemap=synthetic_sky())
    return cfg.settings
