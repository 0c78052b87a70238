"""ctypes mirror of include/halogen_abi.h and a thin, error-checked wrapper around libhalogen_hip.so.

The structs below are byte-identical to the reference's C# blittable structs
(Assets/Scripts/Render Features/HalogenRenderPass.cs:10-76); test_abi.py checks every size and offset
against the header.  There is no fallback: if the shared library is missing, importing `lib()` raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
# HALOGEN_LIB selects an alternative build of the same library (A/B variants in tools/sweep.sh)
LIB_PATH = Path(os.environ["HALOGEN_LIB"]) if os.environ.get("HALOGEN_LIB") else _HERE / "libhalogen_hip.so"


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Vec4(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("w", C.c_float)]


class Mat4(C.Structure):
    """UnityEngine.Matrix4x4 field order (m00, m10, m20, m30, m01, ...): column-major."""

    _fields_ = [("m", C.c_float * 16)]


class HalogenSphere(C.Structure):  # RP:10-19, 44 B
    _fields_ = [("center", Vec3), ("radius", C.c_float), ("materialIndex", C.c_uint32),
                ("boundingCornerA", Vec3), ("boundingCornerB", Vec3)]


class HalogenMeshData(C.Structure):  # RP:21-34, 164 B
    _fields_ = [("triangleBufferOffset", C.c_uint32), ("accelerationBufferOffset", C.c_uint32),
                ("boundingCornerA", Vec3), ("boundingCornerB", Vec3), ("materialIndex", C.c_uint32),
                ("worldToLocal", Mat4), ("localToWorld", Mat4)]


class PackedRayMedium(C.Structure):  # RP:36-42, 24 B
    _fields_ = [("indexOfRefraction", C.c_float), ("absorption", Vec3), ("priority", C.c_int32),
                ("materialID", C.c_uint32)]


class PackedHalogenMaterial(C.Structure):  # RP:44-55, 84 B
    _fields_ = [("materialID", C.c_uint32), ("albedo", Vec4), ("specularAlbedo", Vec4), ("metallic", C.c_float),
                ("roughness", C.c_float), ("emissive", Vec4), ("rayMedium", PackedRayMedium)]


class HalogenTriangle(C.Structure):  # RP:57-66, 72 B
    _fields_ = [("pointA", Vec3), ("pointB", Vec3), ("pointC", Vec3), ("normalA", Vec3), ("normalB", Vec3),
                ("normalC", Vec3)]


class BVHEntry(C.Structure):  # RP:68-76, 32 B
    _fields_ = [("indexA", C.c_uint32), ("triangleCount", C.c_uint32), ("boundingCornerA", Vec3),
                ("boundingCornerB", Vec3)]


class HgParams(C.Structure):  # every uniform of HalgoenCompute.compute:26-68,185
    _fields_ = [
        ("camLocalToWorld", Mat4), ("screenParameters", Vec4), ("viewParameters", Vec4),
        ("cameraParameters", Vec4), ("frameCount", C.c_int32), ("samplesPerPixel", C.c_uint32),
        ("maxBounces", C.c_uint32), ("maxDiffuseBounces", C.c_uint32), ("maxGlossyBounces", C.c_uint32),
        ("maxTransmissionBounces", C.c_uint32), ("halogenDebugMode", C.c_uint32),
        ("triangleDebugDisplayRange", C.c_uint32), ("boxDebugDisplayRange", C.c_uint32),
        ("defaultHDRIMipLevel", C.c_int32), ("focalPlaneDistance", C.c_float), ("focalConeAngle", C.c_float),
        ("filterRadius", C.c_float), ("useEnvironmentCubemap", C.c_int32), ("bufferCounts", Vec4),
    ]


class HgCounters(C.Structure):
    _fields_ = [("paths", C.c_uint64), ("rays", C.c_uint64), ("tri_tests", C.c_uint64),
                ("aabb_tests", C.c_uint64), ("mesh_visits", C.c_uint64), ("sphere_tests", C.c_uint64),
                ("hits", C.c_uint64), ("kernel_ms", C.c_double), ("launches", C.c_uint64),
                ("trace_ms", C.c_double), ("trace_launches", C.c_uint64), ("node_rounds", C.c_uint64),
                ("tri_rounds", C.c_uint64), ("last_kernel", C.c_uint64),
                ("trace_cycles", C.c_uint64), ("shade_cycles", C.c_uint64),
                ("shade_detail", C.c_uint64 * 4), ("shade_rounds", C.c_uint64), ("primary_misses", C.c_uint64),
                ("exec_fallbacks", C.c_uint64), ("trace_busy_ms", C.c_double), ("order_faults", C.c_uint64),
                ("scene_uploads", C.c_uint64), ("scene_uploads_skipped", C.c_uint64),
                ("scene_uploads_partial", C.c_uint64), ("scene_uploads_vouched", C.c_uint64),
                ("server_launches", C.c_uint64),
                ("server_frames", C.c_uint64), ("server_refused", C.c_uint64), ("frames_lost", C.c_uint64),
                ("server_ahead", C.c_uint64)]

    def as_dict(self) -> dict:
        return {name: (list(v) if isinstance(v, C.Array) else v)
                for name, v in ((name, getattr(self, name)) for name, _ in self._fields_)}


HG_OK = 0
HG_KERNEL_MEGA, HG_KERNEL_WAVEFRONT, HG_KERNEL_MEGA_REGEN, HG_KERNEL_MEGA_STREAM, HG_KERNEL_MEGA_POOL = 0, 1, 2, 3, 4
HG_KERNEL_AUTO = 5
HG_OPT_KERNEL, HG_OPT_BLOCK, HG_OPT_COUNTERS, HG_OPT_TIMING, HG_OPT_REFILL, HG_OPT_FRAME_SPLIT = 1, 2, 3, 4, 5, 6
HG_OPT_DESCENT_T = 7
HG_OPT_TILE_ORDER = 8
HG_OPT_COALESCE = 9
HG_OPT_READBACK_DEPTH = 10
HG_OPT_READBACK_STREAM = 11
HG_OPT_WAVE_UNITS = 12
HG_OPT_LANE_PICK = 14
HG_OPT_SERVER = 15
HG_OPT_SERVER_IDLE_US = 16
HG_OPT_SERVER_GATE_US = 17
HG_OPT_QUEUE_FILL = 18
HG_OPT_SERVER_AHEAD = 19
HG_E_INVALID, HG_E_HIP, HG_E_NOMEM, HG_E_NOSCENE, HG_E_NOTARGET, HG_E_UNSUPPORTED, HG_E_COMM = -1, -2, -3, -4, -5, -6, -7
HG_E_FRAME_LOST = -8
HG_READBACK_MAX = 16
# display formats of readback_begin(format=...) (include/halogen_abi.h, csrc/hg_pack.h): bytes per pixel and numpy view
HG_DISPLAY_RGBA32F, HG_DISPLAY_RGBA16F, HG_DISPLAY_R11G11B10F = 0, 1, 2
DISPLAY_FORMATS = {"rgba32f": HG_DISPLAY_RGBA32F, "rgba16f": HG_DISPLAY_RGBA16F, "r11g11b10f": HG_DISPLAY_R11G11B10F}
DISPLAY_BPP = {HG_DISPLAY_RGBA32F: 16, HG_DISPLAY_RGBA16F: 8, HG_DISPLAY_R11G11B10F: 4}

# every symbol include/halogen_abi.h declares (test_abi.py checks the .so exports exactly these)
EXPORTS = [
    "hg_abi_version", "hg_create", "hg_destroy", "hg_last_error", "hg_upload_scene", "hg_upload_scene_gen",
    "hg_upload_cubemap",
    "hg_set_params", "hg_resize", "hg_set_tiling", "hg_clear_accumulation", "hg_render", "hg_synchronize",
    "hg_readback", "hg_readback_begin", "hg_readback_end", "hg_readback_begin_format", "hg_readback_end_data",
    "hg_pack_display", "hg_set_accumulation", "hg_copy_tiles_device", "hg_local_tile_count", "hg_get_counters", "hg_reset_counters",
    "hg_set_option", "hg_selftest", "hg_build_blas", "hg_build_blas_mt", "hg_build_blas_sah", "hg_unity_bounds", "hg_pack_triangles",
    "hg_comm_unique_id", "hg_comm_init_rank", "hg_comm_init_all", "hg_comm_gather", "hg_comm_synchronize",
    "hg_comm_readback", "hg_comm_readback_begin", "hg_comm_readback_end", "hg_comm_set_timeout_ms", "hg_comm_transport", "hg_comm_last_error", "hg_comm_destroy",
    "hg_comm_assemble_host",
]
HG_COMM_ID_BYTES = 128
HG_COMM_RCCL, HG_COMM_PEER = 1, 2
HG_SELFTEST_RCP = 1
HG_SELFTEST_BUILD = 2
HG_BUILD_CHECK_EXEC = 1
HG_BUILD_NO_REGEN_ITEMS = 2

_lib = None


def lib() -> C.CDLL:
    """Load libhalogen_hip.so (built in-tree by `make -C halogen-pathtracer_amd`).  Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} not built: run `make -C halogen-pathtracer_amd` (no CPU fallback exists)")
    L = C.CDLL(str(LIB_PATH))
    P = C.c_void_p
    i32, i64, sz, f32p = C.c_int32, C.c_int64, C.c_size_t, C.POINTER(C.c_float)
    sig = {
        "hg_abi_version": (C.c_int, []),
        "hg_create": (C.c_int, [C.c_int, C.POINTER(P)]),
        "hg_destroy": (None, [P]),
        "hg_last_error": (C.c_char_p, [P]),
        "hg_upload_scene": (C.c_int, [P, P, i32, P, i32, P, i32, P, i32, P, i32]),
        "hg_upload_scene_gen": (C.c_int, [P, C.c_uint64, P, i32, P, i32, P, i32, P, i32, P, i32]),
        "hg_upload_cubemap": (C.c_int, [P, i32, i32, P, sz]),
        "hg_set_params": (C.c_int, [P, C.POINTER(HgParams)]),
        "hg_resize": (C.c_int, [P, i32, i32]),
        "hg_set_tiling": (C.c_int, [P, i32, i32]),
        "hg_clear_accumulation": (C.c_int, [P]),
        "hg_render": (C.c_int, [P, i32, i32]),
        "hg_synchronize": (C.c_int, [P]),
        "hg_readback": (C.c_int, [P, f32p, sz]),
        "hg_readback_begin": (C.c_int, [P]),
        "hg_readback_end": (C.c_int, [P, C.POINTER(f32p), C.POINTER(sz)]),
        "hg_readback_begin_format": (C.c_int, [P, i32]),
        "hg_readback_end_data": (C.c_int, [P, C.POINTER(P), C.POINTER(sz), C.POINTER(i32)]),
        "hg_pack_display": (C.c_int, [f32p, sz, i32, P]),
        "hg_set_accumulation": (C.c_int, [P, f32p, sz, i32]),
        "hg_copy_tiles_device": (C.c_int, [P, P, sz]),
        "hg_local_tile_count": (i32, [P]),
        "hg_get_counters": (C.c_int, [P, C.POINTER(HgCounters)]),
        "hg_reset_counters": (C.c_int, [P]),
        "hg_set_option": (C.c_int, [P, i32, i32]),
        "hg_selftest": (i64, [P, i32, C.POINTER(i64)]),
        "hg_build_blas": (i64, [P, i32, P, i32, f32p, f32p, i32, P, i64]),
        "hg_build_blas_mt": (i64, [P, i32, P, i32, f32p, f32p, i32, P, i64, i32]),
        "hg_build_blas_sah": (i64, [P, i32, P, i32, i32, i32, P, i64]),
        "hg_unity_bounds": (None, [f32p, f32p, i32, f32p, f32p]),
        "hg_pack_triangles": (C.c_int, [P, P, i32, P, i32, P]),
        "hg_comm_unique_id": (C.c_int, [C.c_char_p]),
        "hg_comm_init_rank": (C.c_int, [P, i32, C.c_char_p, i32, C.POINTER(P)]),
        "hg_comm_init_all": (C.c_int, [C.POINTER(P), i32, C.POINTER(P)]),
        "hg_comm_gather": (C.c_int, [P, i32]),
        "hg_comm_synchronize": (C.c_int, [P]),
        "hg_comm_readback": (C.c_int, [P, f32p, sz]),
        "hg_comm_readback_begin": (C.c_int, [P, i32]),
        "hg_comm_readback_end": (C.c_int, [P, C.POINTER(P), C.POINTER(sz), C.POINTER(i32)]),
        "hg_comm_set_timeout_ms": (C.c_int, [P, i64]),
        "hg_comm_assemble_host": (C.c_int, [f32p, i64, i32, i32, i32, f32p, sz]),
        "hg_comm_transport": (C.c_int, [P]),
        "hg_comm_last_error": (C.c_char_p, [P]),
        "hg_comm_destroy": (None, [P]),
    }
    for name, (res, args) in sig.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            if not os.environ.get("HALOGEN_LIB"):
                raise
            continue  # an older A/B build (tools/sweeps) without this entry point
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


class HalogenError(RuntimeError):
    def __init__(self, msg: str, rc: int = 0):
        super().__init__(msg)
        self.rc = rc  # the HG_E_* code (0 when not from an entry point)


def _ptr(a) -> C.c_void_p:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return C.c_void_p(a.ctypes.data)
    return C.cast(a, C.c_void_p)


def _display_view(ptr: C.c_void_p, n_bytes: int, fmt: int, w: int, h: int, copy: bool) -> np.ndarray:
    """A display image (hg_readback_end_data) as (h, w, 4) float32 / (h, w, 4) float16 / (h, w) uint32."""
    bpp = DISPLAY_BPP.get(fmt)
    if bpp is None or n_bytes != w * h * bpp:
        raise HalogenError(f"display readback: {n_bytes} bytes of format {fmt} for a {w}x{h} target")
    raw = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(n_bytes,))
    if fmt == HG_DISPLAY_RGBA32F:
        view = raw.view(np.float32).reshape(h, w, 4)
    elif fmt == HG_DISPLAY_RGBA16F:
        view = raw.view(np.float16).reshape(h, w, 4)
    else:
        view = raw.view(np.uint32).reshape(h, w)
    return view.copy() if copy else view


def as_struct_array(struct_type, n: int):
    return (struct_type * max(n, 0))()


class Context:
    """One HIP device + stream (hg_ctx).  Not thread-safe; one per GPU."""

    def __init__(self, device: int = 0):
        L = lib()
        h = C.c_void_p()
        rc = L.hg_create(int(device), C.byref(h))
        if rc != HG_OK:
            raise HalogenError(f"hg_create(device={device}) failed with {rc} (no usable HIP device?)")
        self._h = h
        self.device = device

    def _check(self, rc: int, what: str):
        if rc != HG_OK:
            msg = lib().hg_last_error(self._h)
            raise HalogenError(f"{what} failed ({rc}): {msg.decode() if msg else ''}", rc)

    def close(self):
        if getattr(self, "_h", None):
            lib().hg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # --- API -----------------------------------------------------------------------------------------
    def upload_scene(self, packed, generation: int = 0) -> None:
        """packed: halogen.scene.PackedScene (ctypes arrays of the reference structs).  generation: the caller's
        geometry generation (hg_upload_scene_gen; 0 = compare every array)."""
        self._check(lib().hg_upload_scene_gen(
            self._h, int(generation), _ptr(packed.spheres), len(packed.spheres), _ptr(packed.meshes), len(packed.meshes),
            _ptr(packed.materials), len(packed.materials), _ptr(packed.triangles), len(packed.triangles),
            _ptr(packed.blas), len(packed.blas)), "hg_upload_scene_gen")

    def upload_cubemap(self, face_size: int, n_mips: int, texels: np.ndarray) -> None:
        t = np.ascontiguousarray(texels, dtype=np.float32)
        self._check(lib().hg_upload_cubemap(self._h, face_size, n_mips, _ptr(t), t.size), "hg_upload_cubemap")

    def set_params(self, p: HgParams) -> None:
        self._check(lib().hg_set_params(self._h, C.byref(p)), "hg_set_params")

    def resize(self, w: int, h: int) -> None:
        self._check(lib().hg_resize(self._h, w, h), "hg_resize")

    def set_tiling(self, rank: int, n_ranks: int) -> None:
        self._check(lib().hg_set_tiling(self._h, rank, n_ranks), "hg_set_tiling")

    def clear_accumulation(self) -> None:
        self._check(lib().hg_clear_accumulation(self._h), "hg_clear_accumulation")

    def render(self, n_frames: int, accumulate: bool = True) -> None:
        self._check(lib().hg_render(self._h, int(n_frames), 1 if accumulate else 0), "hg_render")

    def synchronize(self) -> None:
        self._check(lib().hg_synchronize(self._h), "hg_synchronize")

    def readback(self, w: int, h: int, out: np.ndarray | None = None) -> np.ndarray:
        if out is None:
            out = np.zeros((h, w, 4), dtype=np.float32)
        self._check(lib().hg_readback(self._h, out.ctypes.data_as(C.POINTER(C.c_float)), out.size), "hg_readback")
        return out

    def readback_begin(self, fmt: int | None = None) -> None:
        """hg_readback_begin(_format): enqueue the display readback of every frame rendered so far (at most
        HG_OPT_READBACK_DEPTH outstanding), as RGBA32F or another HG_DISPLAY_* format."""
        if fmt is None:
            self._check(lib().hg_readback_begin(self._h), "hg_readback_begin")
        else:
            self._check(lib().hg_readback_begin_format(self._h, int(fmt)), "hg_readback_begin_format")

    def readback_end(self, w: int, h: int, copy: bool = True) -> np.ndarray:
        """hg_readback_end_data: the image of the oldest begun readback, as (h, w, 4) float32 (RGBA32F), (h, w, 4)
        float16 (RGBA16F) or (h, w) uint32 (R11G11B10F).  copy=False returns a view of the context's pinned host image,
        valid until the depth-th readback_begin after the one it came from."""
        ptr, n, fmt = C.c_void_p(), C.c_size_t(0), C.c_int32(-1)
        self._check(lib().hg_readback_end_data(self._h, C.byref(ptr), C.byref(n), C.byref(fmt)), "hg_readback_end_data")
        return _display_view(ptr, n.value, fmt.value, w, h, copy)

    def set_accumulation(self, image: np.ndarray, frame_count: int) -> None:
        """Checkpoint resume (hg_set_accumulation): the (h, w, 4) image hg_readback returned and the FrameCount of
        the next frame."""
        img = np.ascontiguousarray(image, dtype=np.float32)
        self._check(lib().hg_set_accumulation(self._h, img.ctypes.data_as(C.POINTER(C.c_float)), img.size,
                                              int(frame_count)), "hg_set_accumulation")

    def local_tile_count(self) -> int:
        return int(lib().hg_local_tile_count(self._h))

    def copy_tiles_device(self, dst_ptr: int, n_bytes: int) -> None:
        self._check(lib().hg_copy_tiles_device(self._h, C.c_void_p(dst_ptr), n_bytes), "hg_copy_tiles_device")

    def counters(self) -> dict:
        c = HgCounters()
        self._check(lib().hg_get_counters(self._h, C.byref(c)), "hg_get_counters")
        return c.as_dict()

    def reset_counters(self) -> None:
        self._check(lib().hg_reset_counters(self._h), "hg_reset_counters")

    def set_option(self, option: int, value: int) -> None:
        self._check(lib().hg_set_option(self._h, option, value), "hg_set_option")

    def selftest(self, test: int = HG_SELFTEST_RCP) -> tuple[int, int]:
        """(mismatches, inputs tested) of a device arithmetic self-test."""
        tested = C.c_int64(0)
        r = lib().hg_selftest(self._h, test, C.byref(tested))
        if r < 0:
            self._check(int(r), "hg_selftest")
        return int(r), int(tested.value)


def comm_unique_id() -> bytes:
    """A fresh communicator id (hg_comm_unique_id): made once by the root process and sent to every rank."""
    buf = C.create_string_buffer(HG_COMM_ID_BYTES)
    rc = lib().hg_comm_unique_id(buf)
    if rc != HG_OK:
        raise HalogenError(f"hg_comm_unique_id failed ({rc})")
    return buf.raw


class Comm:
    """hg_comm: the multi-GPU gather of the ranks' tiles to a root.  Comm.rank(ctx, n, id, r) joins
    one process's rank (one process per GPU); Comm.all(ctxs) covers every rank of this process.  Destroy it (close)
    before its contexts."""

    def __init__(self, handle: C.c_void_p, ctxs):
        self._h = handle
        self._ctxs = list(ctxs)  # kept alive while the comm exists

    @classmethod
    def rank(cls, ctx: "Context", n_ranks: int, uid: bytes, rank: int) -> "Comm":
        h = C.c_void_p()
        rc = lib().hg_comm_init_rank(ctx._h, n_ranks, uid, rank, C.byref(h))
        if rc != HG_OK:
            msg = lib().hg_last_error(ctx._h)
            raise HalogenError(f"hg_comm_init_rank failed ({rc}): {msg.decode() if msg else ''}")
        return cls(h, [ctx])

    @classmethod
    def all(cls, ctxs) -> "Comm":
        arr = (C.c_void_p * len(ctxs))(*[c._h for c in ctxs])
        h = C.c_void_p()
        rc = lib().hg_comm_init_all(arr, len(ctxs), C.byref(h))
        if rc != HG_OK:
            msg = lib().hg_last_error(ctxs[0]._h)
            raise HalogenError(f"hg_comm_init_all failed ({rc}): {msg.decode() if msg else ''}")
        return cls(h, ctxs)

    def _check(self, rc: int, what: str):
        if rc != HG_OK:
            msg = lib().hg_comm_last_error(self._h)
            raise HalogenError(f"{what} failed ({rc}): {msg.decode() if msg else ''}", rc)

    @property
    def transport(self) -> int:
        return int(lib().hg_comm_transport(self._h))

    def gather(self, root: int = 0) -> None:
        self._check(lib().hg_comm_gather(self._h, root), "hg_comm_gather")

    def synchronize(self) -> None:
        """Wait for this process's part of the last gather, bounded by the deadline (HalogenError on a dead peer)."""
        self._check(lib().hg_comm_synchronize(self._h), "hg_comm_synchronize")

    def set_timeout_ms(self, ms: int) -> None:
        self._check(lib().hg_comm_set_timeout_ms(self._h, int(ms)), "hg_comm_set_timeout_ms")

    def readback(self, w: int, h: int, out: np.ndarray | None = None) -> np.ndarray:
        if out is None:
            out = np.zeros((h, w, 4), dtype=np.float32)
        self._check(lib().hg_comm_readback(self._h, out.ctypes.data_as(C.POINTER(C.c_float)), out.size),
                    "hg_comm_readback")
        return out

    def readback_begin(self, fmt: int = HG_DISPLAY_RGBA32F) -> None:
        """hg_comm_readback_begin: the pipelined display of the last gather's image (into the root context's ring)."""
        self._check(lib().hg_comm_readback_begin(self._h, int(fmt)), "hg_comm_readback_begin")

    def readback_end(self, w: int, h: int, copy: bool = True) -> np.ndarray:
        """hg_comm_readback_end: the oldest begun display image (bounded wait), shaped as Context.readback_end's."""
        ptr, n, fmt = C.c_void_p(), C.c_size_t(0), C.c_int32(-1)
        self._check(lib().hg_comm_readback_end(self._h, C.byref(ptr), C.byref(n), C.byref(fmt)), "hg_comm_readback_end")
        return _display_view(ptr, n.value, fmt.value, w, h, copy)

    def close(self):
        if getattr(self, "_h", None):
            lib().hg_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def assemble_host(slabs: np.ndarray, width: int, height: int, n_ranks: int) -> np.ndarray:
    """hg_comm_assemble_host: (n_ranks, slab_tiles, 64, 4) float32 tiles (slab r = rank r's local tiles) -> the
    (height, width, 4) image, through the mapping the device gather uses (csrc/hg_tiling.h).  Needs no GPU."""
    s = np.ascontiguousarray(slabs, dtype=np.float32)
    if s.ndim != 4 or s.shape[0] != n_ranks or s.shape[2:] != (64, 4):
        raise ValueError(f"slabs must be (n_ranks={n_ranks}, slab_tiles, 64, 4), got {s.shape}")
    out = np.empty((height, width, 4), np.float32)
    fp = C.POINTER(C.c_float)
    rc = lib().hg_comm_assemble_host(s.ctypes.data_as(fp), s.shape[1], width, height, n_ranks, out.ctypes.data_as(fp),
                                     out.size)
    if rc != HG_OK:
        raise HalogenError(f"hg_comm_assemble_host failed ({rc}): slabs {s.shape} for {width}x{height}, {n_ranks} ranks")
    return out


def pack_display(rgba: np.ndarray, fmt: int) -> np.ndarray:
    """hg_pack_display: (..., 4) float32 pixels in a display format on the host, the device's conversion (no GPU):
    (..., 4) float32, (..., 4) float16 or (...) uint32 (R11G11B10F)."""
    a = np.ascontiguousarray(rgba, dtype=np.float32)
    if a.shape[-1] != 4:
        raise ValueError("rgba must have 4 channels")
    n = a.size // 4
    shape = {HG_DISPLAY_RGBA32F: (a.shape, np.float32), HG_DISPLAY_RGBA16F: (a.shape, np.float16),
             HG_DISPLAY_R11G11B10F: (a.shape[:-1], np.uint32)}
    if fmt not in shape:
        raise ValueError(f"unknown display format {fmt}")
    out = np.empty(*shape[fmt])
    rc = lib().hg_pack_display(a.ctypes.data_as(C.POINTER(C.c_float)), n, int(fmt), C.c_void_p(out.ctypes.data))
    if rc != HG_OK:
        raise HalogenError(f"hg_pack_display failed ({rc})")
    return out


def gpu_available() -> bool:
    """True when a HIP device is visible (without initialising torch)."""
    if os.environ.get("HIP_VISIBLE_DEVICES") == "":
        return False
    try:
        L = lib()
    except RuntimeError:
        return False
    h = C.c_void_p()
    if L.hg_create(0, C.byref(h)) != HG_OK:
        return False
    L.hg_destroy(h)
    return True
