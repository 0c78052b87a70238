"""HalogenSettings + HalogenRenderPass — the host-side API surface of the reference, over the C-ABI.

Mirrors Assets/Scripts/Render Features/HalogenRenderFeature.cs:25-67 (settings) and
Assets/Scripts/Render Features/HalogenRenderPass.cs (RP) — the constructor's clamping (RP:154-233),
OnCameraSetup (RP:237-260), ClearAccumulation (RP:262-268), Execute (RP:270-357), DispatchHalogenTrace's
uniform derivation (RP:359-401), Dispose (RP:410-423) and getFrameCount (RP:548).  Unity's
ComputeShader/ComputeBuffer/RTHandle/Blit calls are replaced by the hg_* entry points (abi.Context).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import abi
from .unity import Transform, to_unity_floats

f32 = np.float32

DEBUG_MODES = {"None": 0, "Albedo": 1, "Normal": 2, "RayTriangleTests": 3, "RayBoxTests": 4, "Combined": 5}


@dataclass
class HalogenSettings:
    """Defaults are the values of Assets/URP-HighFidelity-Renderer.asset:51-77."""

    ShowInSceneView: bool = True
    Accumulate: bool = True
    SamplesPerPixel: int = 1
    MaxAccumulatedFrames: int = 16
    UnlimitedSampling: bool = True
    MaxBounces: int = 12
    DiffuseBounces: int = 4
    GlossyBounces: int = 4
    TransmissionBounces: int = 12
    FilterRadius: float = 1.0
    NearPlaneDistance: float = 0.1
    FarPlaneDistance: float = 5000.0
    FocalPlaneDistance: float = 8.18
    ApertureAngle: float = 0.0
    useHDRISky: bool = True
    environmentCubemap: object = None  # halogen.envmap.Cubemap or None
    EnvironmentMipLevel: int = 1
    FirstInteractionOnly: bool = True
    DebugMode: str = "None"
    TriangleDebugDisplayRange: int = 100
    BoxDebugDisplayRange: int = 153


@dataclass
class Camera:
    """The Unity camera the pass renders for: transform, vertical FOV (degrees) and pixel size."""

    transform: Transform = field(default_factory=Transform)
    fieldOfView: float = 60.0
    pixelWidth: int = 256
    pixelHeight: int = 256

    @property
    def aspect(self) -> float:
        return float(f32(self.pixelWidth) / f32(self.pixelHeight))

    def pose(self):
        """What RP:279-293 compares from frame to frame: the WORLD position and rotation (float32)."""
        return (tuple(float(v) for v in self.transform.position), tuple(float(v) for v in self.transform.rotation))


def unity_equals(a, b) -> bool:
    """Vector3.Equals / Quaternion.Equals (RP:280): componentwise float.Equals, i.e. exact ==, with NaN equal to
    NaN and +0 equal to -0 (the reference does not use the approximate == operator)."""
    return len(a) == len(b) and all(x == y or (math.isnan(x) and math.isnan(y)) for x, y in zip(a, b))


def camera_moved(prior, pose) -> bool:
    """RP:279-284: accumulation is cleared when a prior pose exists and its position or rotation differs."""
    return prior is not None and not (unity_equals(prior[0], pose[0]) and unity_equals(prior[1], pose[1]))


def make_params(settings_clamped: dict, camera: Camera, frame_count: int, n_spheres: int, n_meshes: int,
                use_cubemap: bool) -> abi.HgParams:
    """DispatchHalogenTrace, RP:359-401: every uniform, derived in float32 the way the C# code does."""
    s = settings_clamped
    p = abi.HgParams()
    n_clip = f32(s["NearPlaneDistance"])
    deg2rad = f32(math.pi / 180.0)  # Mathf.Deg2Rad
    half = f32(deg2rad * f32(camera.fieldOfView)) * f32(0.5)
    h = f32(math.tan(float(half))) * n_clip  # Mathf.Tan = (float)Math.Tan
    w = f32(camera.aspect) * h
    p.camLocalToWorld.m[:] = to_unity_floats(camera.transform.local_to_world)
    p.screenParameters = abi.Vec4(camera.pixelWidth, camera.pixelHeight, 0.0, 0.0)
    p.viewParameters = abi.Vec4(float(w), float(h), float(n_clip), float(f32(s["FarPlaneDistance"])))
    pos = camera.transform.position
    p.cameraParameters = abi.Vec4(float(pos[0]), float(pos[1]), float(pos[2]), 0.0)
    p.frameCount = frame_count if s["Accumulate"] else 1
    p.samplesPerPixel = s["SamplesPerPixel"]
    p.maxBounces = s["MaxBounces"]
    p.maxDiffuseBounces = s["MaxDiffuseBounces"]
    p.maxGlossyBounces = s["MaxGlossyBounces"]
    p.maxTransmissionBounces = s["MaxTransmissionBounces"]
    p.halogenDebugMode = s["HalogenDebugMode"]
    p.triangleDebugDisplayRange = s["TriangleDebugDisplayRange"]
    p.boxDebugDisplayRange = s["BoxDebugDisplayRange"]
    p.defaultHDRIMipLevel = s["EnvironmentMipLevel"]
    p.focalPlaneDistance = s["FocalPlaneDistance"]
    p.focalConeAngle = s["ApertureAngle"]
    p.filterRadius = s["FilterRadius"]
    p.useEnvironmentCubemap = 1 if use_cubemap else 0
    p.bufferCounts = abi.Vec4(n_spheres, n_meshes, 0.0, 0.0)
    return p


def clamp_settings(st: HalogenSettings) -> dict:
    """The constructor's clamping and debug-mode mapping, RP:169-231."""
    eps = 1.401298464324817e-45  # Mathf.Epsilon (smallest denormal float)
    d = {}
    d["SamplesPerPixel"] = max(1, int(st.SamplesPerPixel))
    d["MaxBounces"] = max(0, int(st.MaxBounces))
    d["MaxDiffuseBounces"] = max(0, int(st.DiffuseBounces))
    d["MaxGlossyBounces"] = max(0, int(st.GlossyBounces))
    d["MaxTransmissionBounces"] = max(0, int(st.TransmissionBounces))
    d["FilterRadius"] = max(0.0, float(st.FilterRadius))
    d["FocalPlaneDistance"] = max(eps, float(st.FocalPlaneDistance))
    d["NearPlaneDistance"] = max(eps, float(st.NearPlaneDistance))
    d["FarPlaneDistance"] = max(float(f32(d["NearPlaneDistance"]) + f32(eps)), float(st.FarPlaneDistance))
    d["ApertureAngle"] = min(max(float(st.ApertureAngle), 0.0), 89.9)
    d["EnvironmentMipLevel"] = min(max(int(st.EnvironmentMipLevel), 0), 2)
    d["Accumulate"] = bool(st.Accumulate)
    d["MaxAccumulatedFrames"] = max(int(st.MaxAccumulatedFrames), 1)
    d["UnlimitedSampling"] = bool(st.UnlimitedSampling)
    use = bool(st.useHDRISky) and st.environmentCubemap is not None
    d["UseEnvironmentCubemap"] = use
    mode = DEBUG_MODES.get(st.DebugMode, 0) if isinstance(st.DebugMode, str) else int(st.DebugMode)
    d["HalogenDebugMode"] = mode
    if mode != 0 and st.FirstInteractionOnly:
        d["MaxBounces"] = 0
    d["TriangleDebugDisplayRange"] = max(int(st.TriangleDebugDisplayRange), 1)
    d["BoxDebugDisplayRange"] = max(int(st.BoxDebugDisplayRange), 1)
    return d


class HalogenRenderPass:
    """Progressive path tracing of a `halogen.scene.Scene` on one GPU (or one rank's tiles)."""

    def __init__(self, settings: HalogenSettings, device: int = 0, context: abi.Context | None = None):
        self.settings = settings
        self.s = clamp_settings(settings)
        self.ctx = context if context is not None else abi.Context(device)
        # the pass never reads the work counters (the reference has none); off, the render server may trace the next
        # frames of an unchanged camera ahead of the calls (HG_OPT_SERVER_AHEAD)
        self.ctx.set_option(abi.HG_OPT_COUNTERS, 0)
        self.FrameCount = 1
        self.AccumulationBufferDirty = True
        self.ObjectBuffersDirty = True
        self._prior_pose = None
        self._prior_resolution = None
        self._scene_counts = (0, 0)
        self._cubemap_uploaded = False
        # hg_upload_scene_gen's geometry generation: bumped whenever the scene's meshes (cache token, triangle and node
        # counts, in order) differ from the last upload's, so a camera move's re-upload compares only the small arrays
        self._geometry = (None, 0)
        self.rank, self.n_ranks = 0, 1
        # display (RP:343-347): the reference's camera target is R11G11B10 float (URP-HighFidelity.asset:26-27)
        self.display_format = abi.HG_DISPLAY_R11G11B10F
        # frames the shown image lags the traced one: 0, the reference's (it shows the frame it just traced, RP:343-345);
        # set_display(latency=k) opts into showing k frames behind while later frames trace (the C# / C++ passes alike)
        self.display_latency = 0
        self._display_pending = 0
        self._display_resync = False

    # ---- RP:237-268 ----------------------------------------------------------------------------
    def OnCameraSetup(self, width: int, height: int):
        res = (int(width), int(height))
        if res != self._prior_resolution:
            self.ctx.resize(*res)
            self._display_pending = 0  # hg_resize drops the display readbacks in flight
            self.ClearAccumulation()
        self._prior_resolution = res

    def ClearAccumulation(self):
        self.FrameCount = 1
        self.AccumulationBufferDirty = True
        self.ObjectBuffersDirty = True
        # an image from before the clear is never shown: the readbacks in flight are ended unseen, and the next frame
        # is shown as soon as it is traced (the pipeline refills behind it)
        self._drop_display()

    def set_tiling(self, rank: int, n_ranks: int):
        """Multi-GPU: render only the 8x8 tiles t with t % n_ranks == rank (not in the reference)."""
        self.rank, self.n_ranks = rank, n_ranks
        self.ctx.set_tiling(rank, n_ranks)
        self._display_pending = 0
        self.ClearAccumulation()

    def UpdateObjectBuffers(self, scene):
        packed = scene.pack() if hasattr(scene, "pack") else scene
        generation = 0  # a bare PackedScene: every array compared
        if hasattr(scene, "meshes") and hasattr(scene, "pack"):
            sig = tuple((m.cache_token, m.triangle_count, len(m.bvh)) for m in scene.meshes)
            if sig != self._geometry[0]:
                self._geometry = (sig, self._geometry[1] + 1)
            generation = self._geometry[1]
        self.ctx.upload_scene(packed, generation)
        self._scene_counts = (len(packed.spheres), len(packed.meshes))
        cube = self.settings.environmentCubemap
        if self.s["UseEnvironmentCubemap"] and not self._cubemap_uploaded:
            self.ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
            self._cubemap_uploaded = True
        return packed

    # ---- RP:270-357 ----------------------------------------------------------------------------
    def Execute(self, scene, camera: Camera, n_frames: int = 1):
        """One Execute per frame in the reference; n_frames > 1 runs that many frames in ONE dispatch with the
        identical per-frame semantics (FrameCount advancing, same blend) as long as nothing changes between."""
        self.OnCameraSetup(camera.pixelWidth, camera.pixelHeight)
        pose = camera.pose()
        if camera_moved(self._prior_pose, pose):
            self.ClearAccumulation()
        if self.FrameCount > 1 and not self.s["Accumulate"]:
            self.ClearAccumulation()
        self._prior_pose = pose
        if self.ObjectBuffersDirty:
            self.UpdateObjectBuffers(scene)
            self.ObjectBuffersDirty = False
        if not self.s["UnlimitedSampling"] and self.FrameCount > self.s["MaxAccumulatedFrames"]:
            return  # rendering done: the reference only re-blits the finished image
        if not self.s["UnlimitedSampling"]:
            n_frames = min(n_frames, self.s["MaxAccumulatedFrames"] - self.FrameCount + 1)
        p = make_params(self.s, camera, self.FrameCount, *self._scene_counts, self.s["UseEnvironmentCubemap"])
        self.ctx.set_params(p)
        if self.AccumulationBufferDirty:
            self.ctx.clear_accumulation()
            self.AccumulationBufferDirty = False
        self.ctx.render(n_frames, accumulate=self.s["Accumulate"])
        if self.s["Accumulate"]:
            self.FrameCount += n_frames

    # ---- the per-frame display (RP:343-347), pipelined, as the C# and C++ passes do it ---------------------------------
    def set_display(self, fmt: int = abi.HG_DISPLAY_R11G11B10F, latency: int = 0):
        """Display format (abi.HG_DISPLAY_*) and how many frames the shown image may lag (0 .. HG_READBACK_MAX - 1 =
        15; 0, the default, shows each frame before the next is traced, as the reference does)."""
        if not 0 <= latency < abi.HG_READBACK_MAX:
            raise ValueError("display latency out of range")
        self.flush_display()
        self.ctx.set_option(abi.HG_OPT_READBACK_DEPTH, latency + 1)
        self.display_format, self.display_latency = int(fmt), int(latency)

    def display(self):
        """Enqueue the display readback of every frame rendered so far; return the image of `display_latency` calls ago
        (None while the pipeline fills): (h, w) uint32 R11G11B10F, (h, w, 4) float16 or float32."""
        self.ctx.readback_begin(self.display_format)
        self._display_pending += 1
        if self._display_resync:  # the first frame after a clear: shown at once
            self._display_resync = False
            return self.flush_display()
        if self._display_pending <= self.display_latency:
            return None
        self._display_pending -= 1
        w, h = self._prior_resolution
        return self.ctx.readback_end(w, h)

    def _drop_display(self):
        if self._display_pending:
            self.flush_display()  # (ended, not shown)
        self._display_resync = self.display_latency > 0

    def flush_display(self):
        """The newest display image once the readbacks in flight are done (None when none is)."""
        last = None
        w, h = self._prior_resolution or (0, 0)
        while self._display_pending:
            self._display_pending -= 1
            last = self.ctx.readback_end(w, h)
        return last

    def read_image(self) -> np.ndarray:
        w, h = self._prior_resolution
        return self.ctx.readback(w, h)

    def restore(self, image: np.ndarray, frame_count: int):
        """Checkpoint resume (not in the reference, whose resumable state is the accumulation RTHandle and the
        FrameCount field, RP:152,185,347): restore(read_image(), getFrameCount()) on a new pass continues the
        progressive render bit-identically (hg_set_accumulation)."""
        h, w = image.shape[:2]
        self.OnCameraSetup(w, h)
        self.ctx.set_accumulation(image, frame_count)
        self.FrameCount = int(frame_count)
        self.AccumulationBufferDirty = False

    def getFrameCount(self) -> int:
        return self.FrameCount

    def Dispose(self):
        self.ctx.close()
