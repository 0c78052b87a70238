// halogen_render_pass.hpp — the reference's host-side API of the path, in C++ over the C-ABI (halogen_abi.h).
//
// The reference host is C# (Unity): HalogenRenderFeature.cs holds the settings (:25-67) and HalogenRenderPass.cs
// ("RP") drives the compute shader.  There is no C# toolchain in this build's image, so this header restates that
// host surface in C++ with the same names and meanings:
//   HalogenSettings                 HalogenRenderFeature.cs:25-67, defaults URP-HighFidelity-Renderer.asset:51-77
//   clamp_settings                  the constructor's clamping and debug-mode mapping, RP:169-231
//   make_params                     DispatchHalogenTrace's uniform derivation, RP:359-401, in float as C# does it
//   HalogenRenderPass::OnCameraSetup    RP:237-260 (hg_resize on a resolution change)
//   HalogenRenderPass::ClearAccumulation RP:262-268
//   HalogenRenderPass::Execute      RP:270-357 (object buffers, camera-move reset, dispatch + accumulation blit)
//   HalogenRenderPass::Dispose      RP:410-423
//   HalogenRenderPass::getFrameCount RP:548
// Unity's ComputeShader / ComputeBuffer / RTHandle / Blit calls are the hg_* entry points.  The reference has no
// error channel; here a failing entry point throws HalogenError with the library's message (the Python mirror,
// halogen/render_pass.py, raises the same way).  tests/test_host_cpp.py checks make_params against the Python
// mirror byte for byte, and renders through this class on the GPU against the oracle's golden images.
#pragma once

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "halogen_abi.h"

namespace halogen {

class HalogenError : public std::runtime_error {
   public:
    using std::runtime_error::runtime_error;
};

enum class HalogenDebugMode : int32_t { None = 0, Albedo = 1, Normal = 2, RayTriangleTests = 3, RayBoxTests = 4,
                                         Combined = 5 };

// RGBA32F cubemap, layout [mip][face][y][x][4] (hg_upload_cubemap)
struct Cubemap {
    int32_t face_size = 0, n_mips = 0;
    std::vector<float> texels;
};

// HalogenRenderFeature.HalogenSettings (:25-67); defaults of URP-HighFidelity-Renderer.asset:51-77
struct HalogenSettings {
    bool ShowInSceneView = true;
    bool Accumulate = true;
    int32_t SamplesPerPixel = 1;
    int32_t MaxAccumulatedFrames = 16;
    bool UnlimitedSampling = true;
    int32_t MaxBounces = 12;
    int32_t DiffuseBounces = 4;
    int32_t GlossyBounces = 4;
    int32_t TransmissionBounces = 12;
    float FilterRadius = 1.0f;
    float NearPlaneDistance = 0.1f;
    float FarPlaneDistance = 5000.0f;
    float FocalPlaneDistance = 8.18f;
    float ApertureAngle = 0.0f;
    bool useHDRISky = true;
    const Cubemap* environmentCubemap = nullptr;
    int32_t EnvironmentMipLevel = 1;
    bool FirstInteractionOnly = true;
    HalogenDebugMode DebugMode = HalogenDebugMode::None;
    int32_t TriangleDebugDisplayRange = 100;
    int32_t BoxDebugDisplayRange = 153;
};

// What RP reads from the Unity camera: transform.localToWorldMatrix (RP:366), transform.position (RP:369),
// fieldOfView (degrees, vertical), pixelWidth / pixelHeight, aspect.
struct Camera {
    hg_mat4 localToWorld{};  // UnityEngine.Matrix4x4 field order (column-major)
    hg_vec3 position{};      // transform.position (world)
    hg_vec4 rotation{0.0f, 0.0f, 0.0f, 1.0f};  // transform.rotation (world quaternion x, y, z, w)
    float fieldOfView = 60.0f;
    int32_t pixelWidth = 256, pixelHeight = 256;
    float aspect() const { return float(pixelWidth) / float(pixelHeight); }
};

// Vector3.Equals / Quaternion.Equals as RP:280 uses them: componentwise float.Equals, i.e. exact ==, with NaN equal
// to NaN (and +0 equal to -0).  The reference compares the world position and rotation only, so a scale-only change
// or a matrix that differs in its bits but not in those does not clear the accumulation.
inline bool unity_equals(float a, float b) { return a == b || (a != a && b != b); }
inline bool camera_moved(const hg_vec3& p0, const hg_vec4& r0, const Camera& cam) {  // RP:279-284
    const hg_vec3& p = cam.position;
    const hg_vec4& r = cam.rotation;
    const bool same = unity_equals(p0.x, p.x) && unity_equals(p0.y, p.y) && unity_equals(p0.z, p.z) &&
                      unity_equals(r0.x, r.x) && unity_equals(r0.y, r.y) && unity_equals(r0.z, r.z) &&
                      unity_equals(r0.w, r.w);
    return !same;
}

// The settings after the constructor's clamping (RP:169-231)
struct ClampedSettings {
    int32_t SamplesPerPixel, MaxBounces, MaxDiffuseBounces, MaxGlossyBounces, MaxTransmissionBounces;
    float FilterRadius, FocalPlaneDistance, NearPlaneDistance, FarPlaneDistance, ApertureAngle;
    int32_t EnvironmentMipLevel;
    bool Accumulate;
    int32_t MaxAccumulatedFrames;
    bool UnlimitedSampling, UseEnvironmentCubemap;
    int32_t HalogenDebugMode, TriangleDebugDisplayRange, BoxDebugDisplayRange;
};

inline ClampedSettings clamp_settings(const HalogenSettings& st) {
    const float eps = FLT_TRUE_MIN;  // Mathf.Epsilon
    ClampedSettings d{};
    d.SamplesPerPixel = std::max(1, st.SamplesPerPixel);
    d.MaxBounces = std::max(0, st.MaxBounces);
    d.MaxDiffuseBounces = std::max(0, st.DiffuseBounces);
    d.MaxGlossyBounces = std::max(0, st.GlossyBounces);
    d.MaxTransmissionBounces = std::max(0, st.TransmissionBounces);
    d.FilterRadius = std::max(0.0f, st.FilterRadius);
    d.FocalPlaneDistance = std::max(eps, st.FocalPlaneDistance);
    d.NearPlaneDistance = std::max(eps, st.NearPlaneDistance);
    d.FarPlaneDistance = std::max(d.NearPlaneDistance + eps, st.FarPlaneDistance);
    d.ApertureAngle = std::min(std::max(st.ApertureAngle, 0.0f), 89.9f);
    d.EnvironmentMipLevel = std::min(std::max(st.EnvironmentMipLevel, 0), 2);
    d.Accumulate = st.Accumulate;
    d.MaxAccumulatedFrames = std::max(st.MaxAccumulatedFrames, 1);
    d.UnlimitedSampling = st.UnlimitedSampling;
    d.UseEnvironmentCubemap = st.useHDRISky && st.environmentCubemap != nullptr;
    d.HalogenDebugMode = int32_t(st.DebugMode);
    if (d.HalogenDebugMode != 0 && st.FirstInteractionOnly) d.MaxBounces = 0;
    d.TriangleDebugDisplayRange = std::max(st.TriangleDebugDisplayRange, 1);
    d.BoxDebugDisplayRange = std::max(st.BoxDebugDisplayRange, 1);
    return d;
}

// DispatchHalogenTrace, RP:359-401: every uniform, in float (Mathf.Tan = (float)Math.Tan((double)x))
inline hg_params make_params(const ClampedSettings& s, const Camera& cam, int32_t frame_count, int32_t n_spheres,
                             int32_t n_meshes, bool use_cubemap) {
    hg_params p{};
    const float n_clip = s.NearPlaneDistance;
    const float deg2rad = float(3.14159265358979323846 / 180.0);  // Mathf.Deg2Rad
    const float half = (deg2rad * cam.fieldOfView) * 0.5f;
    const float h = float(std::tan(double(half))) * n_clip;
    const float w = cam.aspect() * h;
    p.camLocalToWorld = cam.localToWorld;
    p.screenParameters = hg_vec4{float(cam.pixelWidth), float(cam.pixelHeight), 0.0f, 0.0f};
    p.viewParameters = hg_vec4{w, h, n_clip, s.FarPlaneDistance};
    p.cameraParameters = hg_vec4{cam.position.x, cam.position.y, cam.position.z, 0.0f};
    p.frameCount = s.Accumulate ? frame_count : 1;
    p.samplesPerPixel = uint32_t(s.SamplesPerPixel);
    p.maxBounces = uint32_t(s.MaxBounces);
    p.maxDiffuseBounces = uint32_t(s.MaxDiffuseBounces);
    p.maxGlossyBounces = uint32_t(s.MaxGlossyBounces);
    p.maxTransmissionBounces = uint32_t(s.MaxTransmissionBounces);
    p.halogenDebugMode = uint32_t(s.HalogenDebugMode);
    p.triangleDebugDisplayRange = uint32_t(s.TriangleDebugDisplayRange);
    p.boxDebugDisplayRange = uint32_t(s.BoxDebugDisplayRange);
    p.defaultHDRIMipLevel = s.EnvironmentMipLevel;
    p.focalPlaneDistance = s.FocalPlaneDistance;
    p.focalConeAngle = s.ApertureAngle;
    p.filterRadius = s.FilterRadius;
    p.useEnvironmentCubemap = use_cubemap ? 1 : 0;
    p.bufferCounts = hg_vec4{float(n_spheres), float(n_meshes), 0.0f, 0.0f};
    return p;
}

// The object buffers UpdateObjectBuffers builds (RP:448-509), already packed in the reference's layouts (by the
// engine's C# producers, or by hg_build_blas / hg_pack_triangles and the caller's own material table)
struct SceneBuffers {
    std::vector<HalogenSphere> spheres;
    std::vector<HalogenMeshData> meshes;
    std::vector<PackedHalogenMaterial> materials;
    std::vector<HalogenTriangle> triangles;
    std::vector<BVHEntry> blas;
    // The producer's geometry generation (hg_upload_scene_gen): bump it whenever `triangles` / `blas` change; while it
    // stays the same (non-zero), a re-upload (every camera move, RP:262-268) compares only the small arrays.  0: compare
    // everything.
    uint64_t geometry_generation = 0;
};

class HalogenRenderPass {
   public:
    // RP:154-233: settings are clamped once, as the constructor does
    explicit HalogenRenderPass(const HalogenSettings& settings, int device = 0)
        : settings_(settings), s_(clamp_settings(settings)) {
        check(hg_create(device, &ctx_), "hg_create");
        // the pass never reads the work counters (the reference has none); off, the render server may trace the next
        // frames of an unchanged camera ahead of the calls (HG_OPT_SERVER_AHEAD): a per-frame display stops waiting
        // on each frame's trace
        check(hg_set_option(ctx_, HG_OPT_COUNTERS, 0), "hg_set_option(HG_OPT_COUNTERS)");
    }
    // The library's work counters (Counters()) on or off (off by default in the pass)
    void SetCounters(bool on) { check(hg_set_option(ctx_, HG_OPT_COUNTERS, on ? 1 : 0), "hg_set_option(HG_OPT_COUNTERS)"); }
    HalogenRenderPass(const HalogenRenderPass&) = delete;
    HalogenRenderPass& operator=(const HalogenRenderPass&) = delete;
    ~HalogenRenderPass() { Dispose(); }

    // RP:237-260: a new resolution reallocates (and clears) the accumulation target
    void OnCameraSetup(int32_t width, int32_t height) {
        if (width != prior_w_ || height != prior_h_) {
            check(hg_resize(ctx_, width, height), "hg_resize");
            display_pending_ = 0;  // hg_resize drops the display readbacks in flight
            ClearAccumulation();
        }
        prior_w_ = width;
        prior_h_ = height;
    }

    // RP:262-268.  An image from before the clear is never shown: the display readbacks in flight are ended unseen, and
    // the next frame is shown as soon as it is traced (the pipeline refills behind it).
    void ClearAccumulation() {
        FrameCount = 1;
        AccumulationBufferDirty = true;
        ObjectBuffersDirty = true;
        if (display_pending_ > 0) (void)FlushDisplay();
        display_resync_ = display_latency_ > 0;
    }

    // Multi-GPU (not in the reference): this pass renders only the 8x8 tiles t with t % n_ranks == rank
    void SetTiling(int32_t rank, int32_t n_ranks) {
        check(hg_set_tiling(ctx_, rank, n_ranks), "hg_set_tiling");
        display_pending_ = 0;  // the new tiling drops the display readbacks in flight
        ClearAccumulation();
    }

    // RP:448-509 (the buffers are copied, SetBufferData semantics)
    void UpdateObjectBuffers(const SceneBuffers& sc) {
        check(hg_upload_scene_gen(ctx_, sc.geometry_generation, sc.spheres.data(), int32_t(sc.spheres.size()),
                                  sc.meshes.data(), int32_t(sc.meshes.size()), sc.materials.data(),
                                  int32_t(sc.materials.size()), sc.triangles.data(), int32_t(sc.triangles.size()),
                                  sc.blas.data(), int32_t(sc.blas.size())),
              "hg_upload_scene_gen");
        n_spheres_ = int32_t(sc.spheres.size());
        n_meshes_ = int32_t(sc.meshes.size());
        if (s_.UseEnvironmentCubemap && !cubemap_uploaded_) {
            const Cubemap& c = *settings_.environmentCubemap;
            check(hg_upload_cubemap(ctx_, c.face_size, c.n_mips, c.texels.data(), c.texels.size()),
                  "hg_upload_cubemap");
            cubemap_uploaded_ = true;
        }
    }

    // RP:270-357.  One Execute per frame in the reference; n_frames > 1 runs that many frames in one dispatch with
    // the identical per-frame semantics (FrameCount advancing, the same blend) as long as nothing changes between.
    void Execute(const SceneBuffers& scene, const Camera& camera, int32_t n_frames = 1) {
        OnCameraSetup(camera.pixelWidth, camera.pixelHeight);
        if (have_pose_ && camera_moved(prior_position_, prior_rotation_, camera)) ClearAccumulation();
        if (FrameCount > 1 && !s_.Accumulate) ClearAccumulation();
        prior_position_ = camera.position;
        prior_rotation_ = camera.rotation;
        have_pose_ = true;
        if (ObjectBuffersDirty) {
            UpdateObjectBuffers(scene);
            ObjectBuffersDirty = false;
        }
        if (!s_.UnlimitedSampling && FrameCount > s_.MaxAccumulatedFrames) return;  // finished: only re-blit
        if (!s_.UnlimitedSampling) n_frames = std::min(n_frames, s_.MaxAccumulatedFrames - FrameCount + 1);
        const hg_params p = make_params(s_, camera, FrameCount, n_spheres_, n_meshes_, s_.UseEnvironmentCubemap);
        check(hg_set_params(ctx_, &p), "hg_set_params");
        if (AccumulationBufferDirty) {
            check(hg_clear_accumulation(ctx_), "hg_clear_accumulation");
            AccumulationBufferDirty = false;
        }
        check(hg_render(ctx_, n_frames, s_.Accumulate ? 1 : 0), "hg_render");
        if (s_.Accumulate) FrameCount += n_frames;
    }

    // The reference's per-frame display (RP:343-347: the accumulation target blitted into the URP camera colour target,
    // an R11G11B10 HDR target under URP-HighFidelity.asset:26-27) as a host image, pipelined: Display() enqueues the
    // display readback of every frame rendered so far in the display format and returns the image of `latency` calls
    // ago (an empty image while the pipeline fills), so the next Execute traces while that image crosses PCIe.  The
    // default latency is 0: each frame's image before the next is traced, as the reference shows it (RP:343-345).
    // FlushDisplay() waits for the readbacks in flight and returns the newest image.  The pointer stays valid until
    // the next Display / FlushDisplay / OnCameraSetup with a new size.
    struct DisplayImage {
        const void* data = nullptr;
        size_t bytes = 0;
        int32_t format = HG_DISPLAY_R11G11B10F;
    };
    // format: HG_DISPLAY_R11G11B10F (the reference's camera target, 4 B/px), HG_DISPLAY_RGBA16F or HG_DISPLAY_RGBA32F;
    // latency: 0 (each image before the next frame is traced) .. HG_READBACK_MAX - 1 frames behind
    void SetDisplay(int32_t format, int32_t latency) {
        if (latency < 0 || latency >= HG_READBACK_MAX) throw HalogenError("display latency out of range");
        (void)FlushDisplay();
        check(hg_set_option(ctx_, HG_OPT_READBACK_DEPTH, latency + 1), "hg_set_option(HG_OPT_READBACK_DEPTH)");
        display_format_ = format;
        display_latency_ = latency;
    }
    DisplayImage Display() {
        check(hg_readback_begin_format(ctx_, display_format_), "hg_readback_begin_format");
        ++display_pending_;
        if (display_resync_) {  // the first frame after a clear: shown at once
            display_resync_ = false;
            return FlushDisplay();
        }
        if (display_pending_ <= display_latency_) return DisplayImage{};
        return end_display();
    }
    DisplayImage FlushDisplay() {
        DisplayImage last{};
        while (display_pending_ > 0) last = end_display();
        return last;
    }
    int32_t display_format() const { return display_format_; }
    int32_t display_latency() const { return display_latency_; }

    // The accumulated image, row-major RGBA32F (what the reference blits to the camera target); blocks
    std::vector<float> Readback() {
        std::vector<float> img(size_t(prior_w_) * size_t(prior_h_) * 4);
        check(hg_readback(ctx_, img.data(), img.size()), "hg_readback");
        return img;
    }

    // Checkpoint / resume (not in the reference, whose resumable state is the accumulation RTHandle and the FrameCount
    // field, RP:152,185,347): Restore(Readback(), getFrameCount()) on a new pass of the same width x height continues
    // the progressive render bit-identically (hg_set_accumulation).
    void Restore(const std::vector<float>& image, int32_t width, int32_t height, int32_t frame_count) {
        OnCameraSetup(width, height);
        check(hg_set_accumulation(ctx_, image.data(), image.size(), frame_count), "hg_set_accumulation");
        FrameCount = frame_count;
        AccumulationBufferDirty = false;
    }

    hg_counters Counters() const {
        hg_counters c{};
        check(hg_get_counters(ctx_, &c), "hg_get_counters");
        return c;
    }

    // RP:410-423
    void Dispose() {
        if (ctx_) hg_destroy(ctx_);
        ctx_ = nullptr;
    }

    // RP:548
    int32_t getFrameCount() const { return FrameCount; }

    const ClampedSettings& clamped() const { return s_; }
    hg_ctx* context() const { return ctx_; }

    int32_t FrameCount = 1;
    bool AccumulationBufferDirty = true;
    bool ObjectBuffersDirty = true;

   private:
    DisplayImage end_display() {
        DisplayImage d;
        check(hg_readback_end_data(ctx_, &d.data, &d.bytes, &d.format), "hg_readback_end_data");
        --display_pending_;
        return d;
    }
    void check(int rc, const char* what) const {
        if (rc != HG_OK) {
            const char* msg = ctx_ ? hg_last_error(ctx_) : nullptr;
            throw HalogenError(std::string(what) + " failed (" + std::to_string(rc) + "): " + (msg ? msg : ""));
        }
    }

    HalogenSettings settings_;
    ClampedSettings s_;
    hg_ctx* ctx_ = nullptr;
    int32_t display_format_ = HG_DISPLAY_R11G11B10F, display_latency_ = 0, display_pending_ = 0;
    bool display_resync_ = false;
    int32_t prior_w_ = -1, prior_h_ = -1;
    hg_vec3 prior_position_{};  // PriorCameraPosition / PriorCameraRotation (RP:293-294)
    hg_vec4 prior_rotation_{};
    bool have_pose_ = false;
    int32_t n_spheres_ = 0, n_meshes_ = 0;
    bool cubemap_uploaded_ = false;
};

}  // namespace halogen
