"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/hg_oracle.c).

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The oracle is the parity
checker and the CPU baseline; the product path never touches it.  PARITY UNPINNED against reference outputs
(the reference has none and cannot run here) — see oracle/hg_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "libhgoracle.so"
# the stats build (HGO_STATS=1): the same oracle with the traversal diagnostics compiled in (stack_stats, visit_stats);
# the plain build above has none of them in its traversal loop (it is the parity checker and the CPU baseline)
LIB_STATS = HERE / "build" / "libhgoracle_stats.so"


class HgoScene(C.Structure):
    _fields_ = [("spheres", C.c_void_p), ("n_spheres", C.c_int32), ("meshes", C.c_void_p), ("n_meshes", C.c_int32),
                ("materials", C.c_void_p), ("n_materials", C.c_int32), ("triangles", C.c_void_p),
                ("n_triangles", C.c_int32), ("blas", C.c_void_p), ("n_nodes", C.c_int32),
                ("cube_texels", C.c_void_p), ("cube_face_size", C.c_int32), ("cube_mips", C.c_int32)]


_libs: dict = {}


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib(stats: bool = False):
    """The plain oracle, or (stats=True) its stats build."""
    path = LIB_STATS if stats else LIB
    if path not in _libs:
        if not path.exists():
            build()
        L = C.CDLL(str(path))
        u32 = C.c_uint32
        L.hgo_pcg_hash.restype = u32
        L.hgo_pcg_hash.argtypes = [u32]
        L.hgo_hash_combine.restype = u32
        L.hgo_hash_combine.argtypes = [u32, u32]
        L.hgo_owen_scramble.restype = u32
        L.hgo_owen_scramble.argtypes = [u32, u32]
        L.hgo_sobol1d.restype = u32
        L.hgo_sobol1d.argtypes = [u32, u32]
        L.hgo_sobol_table.restype = u32
        L.hgo_sobol_table.argtypes = [u32, u32]
        L.hgo_u32_owen_scrambled_sobol.restype = u32
        L.hgo_u32_owen_scrambled_sobol.argtypes = [u32, u32, u32]
        L.hgo_u32_2d_owen_scrambled_sobol.restype = None
        L.hgo_u32_2d_owen_scrambled_sobol.argtypes = [u32, u32, u32, C.POINTER(u32)]
        L.hgo_inverted_blackman_harris.restype = C.c_float
        L.hgo_inverted_blackman_harris.argtypes = [C.c_float]
        L.hgo_build_blas.restype = C.c_int64
        L.hgo_build_blas.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.POINTER(C.c_float),
                                     C.POINTER(C.c_float), C.c_int32, C.c_void_p, C.c_int64]
        L.hgo_render.restype = C.c_int
        L.hgo_render.argtypes = [C.POINTER(HgoScene), C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int64,
                                 C.c_int64, C.c_int32, C.c_void_p]
        L.hgo_trace_pixel.restype = None
        L.hgo_trace_pixel.argtypes = [C.POINTER(HgoScene), C.c_void_p, u32, u32, C.c_int32, C.POINTER(C.c_float),
                                      C.c_void_p]
        fp = C.POINTER(C.c_float)
        L.hgo_sphere_t.restype = C.c_float
        L.hgo_sphere_t.argtypes = [fp, fp, fp, C.c_float]
        L.hgo_triangle_t.restype = C.c_float
        L.hgo_triangle_t.argtypes = [fp, fp, fp, fp, fp, fp, fp, fp]
        L.hgo_aabb_t.restype = C.c_float
        L.hgo_aabb_t.argtypes = [fp, fp, fp, fp]
        L.hgo_stack_stats.restype = None
        L.hgo_stack_stats.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_int32), C.c_int32]
        L.hgo_visit_stats.restype = None
        L.hgo_visit_stats.argtypes = [C.POINTER(C.c_uint64), C.c_int32]
        L.hgo_cube_sample.restype = None
        L.hgo_cube_sample.argtypes = [C.POINTER(HgoScene), fp, C.c_int32, fp]
        L.hgo_cube_adjacent.restype = None
        L.hgo_cube_adjacent.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32)]
        L.hgo_stats_build.restype = C.c_int
        L.hgo_stats_build.argtypes = []
        _libs[path] = L
    return _libs[path]


def make_scene(packed, cubemap=None) -> tuple[HgoScene, list]:
    keep = [packed]
    s = HgoScene()
    s.spheres, s.n_spheres = C.cast(packed.spheres, C.c_void_p), len(packed.spheres)
    s.meshes, s.n_meshes = C.cast(packed.meshes, C.c_void_p), len(packed.meshes)
    s.materials, s.n_materials = C.cast(packed.materials, C.c_void_p), len(packed.materials)
    s.triangles, s.n_triangles = C.cast(packed.triangles, C.c_void_p), len(packed.triangles)
    s.blas, s.n_nodes = C.cast(packed.blas, C.c_void_p), len(packed.blas)
    if cubemap is not None:
        tex = np.ascontiguousarray(cubemap.texels, dtype=np.float32)
        keep.append(tex)
        s.cube_texels = tex.ctypes.data
        s.cube_face_size, s.cube_mips = cubemap.face_size, cubemap.n_mips
    return s, keep


class Counters(C.Structure):  # hg_counters layout (include/halogen_abi.h), complete: the oracle writes any field
    _fields_ = [("paths", C.c_uint64), ("rays", C.c_uint64), ("tri_tests", C.c_uint64),
                ("aabb_tests", C.c_uint64), ("mesh_visits", C.c_uint64), ("sphere_tests", C.c_uint64),
                ("hits", C.c_uint64), ("kernel_ms", C.c_double), ("launches", C.c_uint64),
                ("trace_ms", C.c_double), ("trace_launches", C.c_uint64), ("node_rounds", C.c_uint64),
                ("tri_rounds", C.c_uint64), ("last_kernel", C.c_uint64), ("trace_cycles", C.c_uint64),
                ("shade_cycles", C.c_uint64), ("shade_detail", C.c_uint64 * 4), ("shade_rounds", C.c_uint64),
                ("primary_misses", C.c_uint64)]
    _oracle_fields = ("paths", "rays", "tri_tests", "aabb_tests", "mesh_visits", "sphere_tests", "hits",
                      "kernel_ms", "launches", "trace_ms", "trace_launches", "primary_misses")

    def as_dict(self):
        return {n: getattr(self, n) for n in self._oracle_fields}


def render(packed, params, n_frames: int, accumulate: bool = True, acc: np.ndarray | None = None,
           cubemap=None, pix_range=None, threads: int | None = None, stats: bool = False):
    """Render n_frames into acc ((H, W, 4) float32, row-major); returns (acc, counters dict).  stats=True renders
    through the stats build, which also feeds stack_stats() / visit_stats()."""
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    if acc is None:
        acc = np.zeros((H, W, 4), dtype=np.float32)
    scene, keep = make_scene(packed, cubemap)
    cnt = Counters()
    p0, p1 = pix_range if pix_range is not None else (0, W * H)
    threads = threads or min(os.cpu_count() or 1, 64)
    rc = lib(stats).hgo_render(C.byref(scene), C.byref(params), n_frames, 1 if accumulate else 0, acc.ctypes.data, p0, p1,
                          threads, C.byref(cnt))
    if rc != 0:
        raise RuntimeError(f"hgo_render failed: {rc}")
    del keep
    return acc, cnt.as_dict()


def stack_stats(reset: bool = False) -> tuple[int, int]:
    """(mesh traversals whose node stack outgrew the reference's NodeStack[32], deepest stack) since the last reset, over
    the renders made with stats=True."""
    n, d = C.c_uint64(0), C.c_int32(0)
    lib(True).hgo_stack_stats(C.byref(n), C.byref(d), 1 if reset else 0)
    return int(n.value), int(d.value)


def visit_stats(reset: bool = False) -> dict:
    """Inner-node visits by the number of children the exact test keeps (0/1/2), for mesh roots and deeper nodes, over
    the renders made with stats=True."""
    out = (C.c_uint64 * 6)()
    lib(True).hgo_visit_stats(out, 1 if reset else 0)
    return {"root": [int(x) for x in out[:3]], "inner": [int(x) for x in out[3:]]}


def cube_adjacent(face: int, i: int, j: int, size: int) -> tuple[int, int, int]:
    out = (C.c_int32 * 3)()
    lib().hgo_cube_adjacent(face, i, j, size, out)
    return int(out[0]), int(out[1]), int(out[2])


def cube_sample(cubemap, d, level: int) -> np.ndarray:
    s = HgoScene()
    tex = np.ascontiguousarray(cubemap.texels, dtype=np.float32)
    s.cube_texels = tex.ctypes.data
    s.cube_face_size, s.cube_mips = cubemap.face_size, cubemap.n_mips
    dv = (C.c_float * 3)(*[float(x) for x in d])
    rgb = (C.c_float * 3)()
    lib().hgo_cube_sample(C.byref(s), dv, level, rgb)
    return np.array(list(rgb), dtype=np.float32)
