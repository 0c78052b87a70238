"""Host-side scene objects and buffer packing — the mirror of the reference's C# host data producers.

  HalogenMaterial        Assets/Scripts/RayTracingManager.cs:6-38   (authoring struct + defaults)
  RayTracingMesh         Assets/Scripts/RayTracingMesh.cs           (cache mesh data, build BLAS, pack tris)
  RayTracingSphere       Assets/Scripts/RayTracingSphere.cs
  Scene (registry)       Assets/Scripts/RayTracingManager.cs:40-145 (enumeration order = buffer order)
  pack_scene             HalogenRenderPass.UpdateObjectBuffers / PackHalogenMaterial / PackMaterialToList
                         (Render Features/HalogenRenderPass.cs:425-537)

The BLAS build and triangle packing run in the native library (hg_build_blas / hg_pack_triangles,
restating BVHGenerator.cs and RayTracingMesh.UpdateTriangleList); all float32 arithmetic the C# code does
on packed values (1/subsurface * absorption, bounds centre/extents) is done in float32 here as well.
"""
from __future__ import annotations

import ctypes as C
import itertools
import os
from dataclasses import dataclass, field

import numpy as np

from . import abi
from .unity import Transform, mesh_bounds_min_max, to_unity_floats

f32 = np.float32


def _c(v) -> float:
    return float(f32(v))


@dataclass(frozen=True)
class HalogenMaterial:
    """RayTracingManager.cs:6-38.  Colors are linear RGBA (the project uses linear space)."""

    color: tuple = (1.0, 1.0, 1.0, 1.0)
    roughness: float = 1.0
    metallic: float = 0.0
    specularColor: tuple = (1.0, 1.0, 1.0, 1.0)
    subsurfaceColor: tuple = (1.0, 1.0, 1.0, 1.0)
    indexOfRefraction: float = 1.0
    absorption: float = 0.0
    dielectricPriority: int = 0
    emissionColor: tuple = (0.0, 0.0, 0.0, 1.0)  # Color.black
    emissionIntensity: float = 0.0

    def __post_init__(self):  # store exactly what a C# float field would hold
        for name in ("color", "specularColor", "subsurfaceColor", "emissionColor"):
            object.__setattr__(self, name, tuple(_c(v) for v in getattr(self, name)))
        for name in ("roughness", "metallic", "indexOfRefraction", "absorption", "emissionIntensity"):
            object.__setattr__(self, name, _c(getattr(self, name)))
        object.__setattr__(self, "dielectricPriority", int(self.dielectricPriority))

    @staticmethod
    def default(color=(1.0, 1.0, 1.0, 1.0)) -> "HalogenMaterial":
        """new HalogenMaterial(defaultColor): color = specular = subsurface = defaultColor (:24-37)."""
        return HalogenMaterial(color=color, specularColor=color, subsurfaceColor=color)


def pack_material(m: HalogenMaterial, material_id: int) -> abi.PackedHalogenMaterial:
    """PackHalogenMaterial, RP:425-446."""
    p = abi.PackedHalogenMaterial()
    p.materialID = material_id
    p.albedo = abi.Vec4(*m.color)
    p.specularAlbedo = abi.Vec4(*m.specularColor)
    p.metallic = m.metallic
    p.roughness = m.roughness
    p.emissive = abi.Vec4(m.emissionColor[0], m.emissionColor[1], m.emissionColor[2], m.emissionIntensity)
    sub = [f32(v) for v in m.subsurfaceColor[:3]]
    amax = f32(max(m.absorption, 0.0))  # Mathf.Max(material.absorption, 0)
    with np.errstate(divide="ignore", invalid="ignore"):
        absorb = [float((f32(1.0) / s) * amax) for s in sub]  # new Vector3(1/x,1/y,1/z) * max(...)
    p.rayMedium.indexOfRefraction = m.indexOfRefraction
    p.rayMedium.absorption = abi.Vec3(*absorb)
    p.rayMedium.priority = m.dielectricPriority
    p.rayMedium.materialID = material_id
    return p


# BLAS builder of the meshes constructed from here on: "reference" (BVHGenerator.cs, the drop-in's parity path) or
# "sah" (hg_build_blas_sah: a binned-SAH hierarchy in the same format, NOT the reference's images)
BLAS_BUILDERS = ("reference", "sah")
_blas_builder = "reference"
SAH_MAX_LEAF = 2


def set_blas_builder(name: str) -> str:
    """Select the BLAS builder for meshes built afterwards; returns the previous one."""
    global _blas_builder
    if name not in BLAS_BUILDERS:
        raise ValueError(f"unknown BLAS builder {name!r}")
    prev, _blas_builder = _blas_builder, name
    return prev


_CACHE_TOKENS = itertools.count(1)


class RayTracingMesh:
    """RayTracingMesh.cs: submesh-0 triangles, vertices and normals of a mesh + its transform + material.

    CacheRaytracingData (:51-68) runs at construction: the BLAS is built (reordering the triangle list in
    place, exactly as the C# builder does) and the 72-B triangles are packed from the reordered list.
    """

    def __init__(self, name: str, vertices, normals, triangles, transform: Transform,
                 material: HalogenMaterial | None = None, max_hierarchy_depth: int = 32):
        self.name = name
        self.vertices = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
        self.normals = np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 3)
        self.triangles = np.ascontiguousarray(triangles, dtype=np.int32).reshape(-1, 3).copy()
        if self.normals.shape != self.vertices.shape:
            raise ValueError("normals must match vertices")
        self.transform = transform
        self.material = material if material is not None else HalogenMaterial.default()
        self.max_hierarchy_depth = int(max_hierarchy_depth)
        self.blas_builder = _blas_builder
        self._cache()

    def _cache(self):
        # a new token whenever the geometry is (re)cached, as the reference's manager ID is new on every OnEnable
        # (RayTracingManager.cs:74-79): the pass's geometry generation keys on it (id() of a collected mesh is reused)
        self.cache_token = next(_CACHE_TOKENS)
        L = abi.lib()
        n_tris = len(self.triangles)
        mn, mx = mesh_bounds_min_max(self.vertices) if len(self.vertices) else (np.zeros(3, f32), np.zeros(3, f32))
        mn = np.ascontiguousarray(mn, dtype=np.float32)
        mx = np.ascontiguousarray(mx, dtype=np.float32)
        fp = C.POINTER(C.c_float)
        cap = 2 * n_tris + 2
        nodes = (abi.BVHEntry * cap)()
        # the parallel build returns the same nodes and triangle order (tests/test_bvh.py); 8 workers measured
        # best on the GPU box's host (tools/bench_build.py: 871k triangles 0.12 s -> 0.05 s)
        if self.blas_builder == "sah":
            n = L.hg_build_blas_sah(self.vertices.ctypes.data, len(self.vertices), self.triangles.ctypes.data, n_tris,
                                    SAH_MAX_LEAF, 48, C.cast(nodes, C.c_void_p), cap)
        else:
            n = L.hg_build_blas_mt(self.vertices.ctypes.data, len(self.vertices), self.triangles.ctypes.data, n_tris,
                                   mn.ctypes.data_as(fp), mx.ctypes.data_as(fp), self.max_hierarchy_depth,
                                   C.cast(nodes, C.c_void_p), cap, min(8, len(os.sched_getaffinity(0))))
        if n < 0:
            raise abi.HalogenError(f"hg_build_blas failed for {self.name}: {n}")
        self.bvh = (abi.BVHEntry * n)()
        C.memmove(self.bvh, nodes, n * C.sizeof(abi.BVHEntry))
        self.packed_triangles = (abi.HalogenTriangle * n_tris)()
        rc = L.hg_pack_triangles(self.vertices.ctypes.data, self.normals.ctypes.data, len(self.vertices),
                                 self.triangles.ctypes.data, n_tris, C.cast(self.packed_triangles, C.c_void_p))
        if rc != 0:
            raise abi.HalogenError(f"hg_pack_triangles failed for {self.name}: {rc}")

    @property
    def triangle_count(self) -> int:
        return len(self.triangles)

    def world_bounds(self):
        """meshRenderer.bounds padded as GetBounds (:106-117): world AABB of the transformed local box."""
        mn, mx = mesh_bounds_min_max(self.vertices)
        corners = np.array([[x, y, z, 1.0] for x in (mn[0], mx[0]) for y in (mn[1], mx[1]) for z in (mn[2], mx[2])])
        w = (self.transform.local_to_world @ corners.T).T[:, :3]
        return unity_bounds(w.min(axis=0), w.max(axis=0), pad=True)

    def mesh_data(self, material_index: int, tri_offset: int, node_offset: int) -> abi.HalogenMeshData:
        """GetRefreshedMeshData, RayTracingMesh.cs:89-104."""
        d = abi.HalogenMeshData()
        bmin, bmax = self.world_bounds()
        d.boundingCornerA = abi.Vec3(*bmin)
        d.boundingCornerB = abi.Vec3(*bmax)
        d.triangleBufferOffset = tri_offset
        d.accelerationBufferOffset = node_offset
        d.materialIndex = material_index
        d.localToWorld.m[:] = to_unity_floats(self.transform.local_to_world)
        d.worldToLocal.m[:] = to_unity_floats(self.transform.world_to_local)
        return d


class RayTracingSphere:
    """RayTracingSphere.cs: centre = transform.position (world), radius = the serialized field."""

    def __init__(self, name: str, transform: Transform, radius: float, material: HalogenMaterial | None = None):
        self.name = name
        self.transform = transform
        self.radius = _c(radius)
        self.material = material if material is not None else HalogenMaterial.default()


def unity_bounds(mn, mx, pad: bool):
    """UnityEngine.Bounds round trip (SetMinMax -> min/max), optionally with the thin-box pad."""
    fp = C.POINTER(C.c_float)
    a = np.ascontiguousarray(mn, dtype=np.float32)
    b = np.ascontiguousarray(mx, dtype=np.float32)
    o1 = np.zeros(3, np.float32)
    o2 = np.zeros(3, np.float32)
    abi.lib().hg_unity_bounds(a.ctypes.data_as(fp), b.ctypes.data_as(fp), 1 if pad else 0, o1.ctypes.data_as(fp),
                              o2.ctypes.data_as(fp))
    return o1, o2


@dataclass
class PackedScene:
    spheres: object
    meshes: object
    materials: object
    triangles: object
    blas: object
    names: list = field(default_factory=list)

    def counts(self) -> dict:
        return {"spheres": len(self.spheres), "meshes": len(self.meshes), "materials": len(self.materials),
                "triangles": len(self.triangles), "blas": len(self.blas)}

    def as_numpy(self) -> dict:
        """Raw bytes of each buffer (for hashing / fixtures)."""
        return {k: np.frombuffer(bytes(getattr(self, k)), dtype=np.uint8)
                for k in ("spheres", "meshes", "materials", "triangles", "blas")}


class Scene:
    """The RayTracingManager registries: spheres and meshes in enumeration (= buffer) order."""

    def __init__(self):
        self.spheres: list[RayTracingSphere] = []
        self.meshes: list[RayTracingMesh] = []

    def add(self, obj):
        (self.spheres if isinstance(obj, RayTracingSphere) else self.meshes).append(obj)
        return obj

    def pack(self) -> PackedScene:
        """UpdateObjectBuffers, RP:448-509 (with PackMaterialToList's struct-equality dedup, :524-537)."""
        unpacked: list[HalogenMaterial] = []
        materials: list[abi.PackedHalogenMaterial] = []

        def material_index(m: HalogenMaterial) -> int:
            if m in unpacked:
                return unpacked.index(m)
            unpacked.append(m)
            materials.append(pack_material(m, len(materials)))
            return len(materials) - 1

        sph = []
        for s in self.spheres:
            hs = abi.HalogenSphere()
            c = s.transform.position
            r = f32(s.radius)
            hs.center = abi.Vec3(*c)
            hs.radius = float(r)
            hs.materialIndex = material_index(s.material)
            hs.boundingCornerA = abi.Vec3(*(c - np.array([r, r, r], np.float32)))
            hs.boundingCornerB = abi.Vec3(*(c + np.array([r, r, r], np.float32)))
            sph.append(hs)
        mesh_records, tri_chunks, node_chunks = [], [], []
        n_tris = n_nodes = 0
        for m in self.meshes:
            mi = material_index(m.material)
            tri_chunks.append(m.packed_triangles)
            mesh_records.append(m.mesh_data(mi, n_tris, n_nodes))
            node_chunks.append(m.bvh)
            n_tris += m.triangle_count
            n_nodes += len(m.bvh)
        tris = (abi.HalogenTriangle * n_tris)()
        nodes = (abi.BVHEntry * n_nodes)()
        ot = on = 0
        for tc, nc in zip(tri_chunks, node_chunks):
            C.memmove(C.addressof(tris) + ot * C.sizeof(abi.HalogenTriangle), tc, C.sizeof(tc))
            C.memmove(C.addressof(nodes) + on * C.sizeof(abi.BVHEntry), nc, C.sizeof(nc))
            ot += len(tc)
            on += len(nc)
        return PackedScene(
            spheres=(abi.HalogenSphere * len(sph))(*sph),
            meshes=(abi.HalogenMeshData * len(mesh_records))(*mesh_records),
            materials=(abi.PackedHalogenMaterial * len(materials))(*materials),
            triangles=tris,
            blas=nodes,
            names=[s.name for s in self.spheres] + [m.name for m in self.meshes],
        )
