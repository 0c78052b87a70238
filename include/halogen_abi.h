/*
 * halogen_abi.h — the drop-in C-ABI boundary of the Halogen path-tracing hot path on MI355X (gfx950).
 *
 * What it replaces (reference: /root/reference, Unity 2022.3 + URP 14):
 *   The ComputeShader / ComputeBuffer / RTHandle calls inside
 *   `Assets/Scripts/Render Features/HalogenRenderPass.cs` ("RP" below):
 *     - buffer (re)allocation            RP:498-502, RP:539-546  -> hg_upload_scene (copies, owns device memory)
 *     - buffer uploads (SetBufferData)   RP:504-508              -> hg_upload_scene
 *     - cubemap binding                  RP:397-398              -> hg_upload_cubemap
 *     - uniform binding                  RP:360-401              -> hg_set_params
 *     - RTHandle allocation on resize    RP:237-260              -> hg_resize
 *     - ClearAccumulation                RP:262-268, RP:333-338  -> hg_clear_accumulation
 *     - DispatchCompute + accumulation   RP:324-347, RP:406      -> hg_render (trace + fused accumulate)
 *       blit (AccumulationShader.shader:27-34)
 *     - Dispose / Release                RP:410-423              -> hg_destroy
 *   plus what the reference never had: readback, counters, error text, multi-GPU tiling.
 *
 * The host structs below are byte-identical to the reference's C# blittable structs
 * (RP:10-76, strides from Marshal.SizeOf at RP:163-167): a C# caller passes its List<T>.ToArray()
 * unchanged through P/Invoke.  Device-side layouts are private to the library
 * (SoA / child-pair records, repacked inside hg_upload_scene).
 *
 * Conventions:
 *   - every int-returning function returns HG_OK (0) or a negative HG_E_* code; hg_last_error() has text.
 *   - host arrays are copied during the call (SetBufferData semantics); counts of 0 are legal.
 *   - one context = one device + one HIP stream; a context is NOT thread-safe; one context per GPU may be
 *     driven from separate host threads.  hg_render is asynchronous; hg_readback / hg_synchronize block.
 *   - held frames (HG_OPT_COALESCE): hg_render may hold its frames and launch them with later calls; every other entry
 *     point launches the held frames first.  A launch that fails there (out of memory, a HIP error) is reported by
 *     THAT entry point, with the text of the failed launch, and the held frames are lost (FrameCount does not advance
 *     for them).  hg_destroy discards held frames without launching them.
 *   - no torch / HIP types appear in any signature.
 */
#ifndef HALOGEN_ABI_H
#define HALOGEN_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HG_ABI_VERSION 6

/* ----------------------------------------------------------------------------------------------
 * Reference host structs (byte-identical to the C# [Sequential] structs)
 * -------------------------------------------------------------------------------------------- */
typedef struct hg_vec3 { float x, y, z; } hg_vec3;
typedef struct hg_vec4 { float x, y, z, w; } hg_vec4;

/* UnityEngine.Matrix4x4: fields m00,m10,m20,m30,m01,... i.e. column-major; element (r,c) = m[c*4+r].
 * HLSL mul(M, v) in the reference = sum_c M(r,c) * v_c. */
typedef struct hg_mat4 { float m[16]; } hg_mat4;

/* HalogenSphere, RP:10-19 (44 B) */
typedef struct HalogenSphere {
    hg_vec3 center;
    float radius;
    uint32_t materialIndex;
    hg_vec3 boundingCornerA;
    hg_vec3 boundingCornerB;
} HalogenSphere;

/* HalogenMeshData, RP:21-34 (164 B) */
typedef struct HalogenMeshData {
    uint32_t triangleBufferOffset;
    uint32_t accelerationBufferOffset;
    hg_vec3 boundingCornerA;
    hg_vec3 boundingCornerB;
    uint32_t materialIndex;
    hg_mat4 worldToLocal;
    hg_mat4 localToWorld;
} HalogenMeshData;

/* PackedRayMedium, RP:36-42 (24 B) */
typedef struct PackedRayMedium {
    float indexOfRefraction;
    hg_vec3 absorption;
    int32_t priority;
    uint32_t materialID;
} PackedRayMedium;

/* PackedHalogenMaterial, RP:44-55 (84 B) */
typedef struct PackedHalogenMaterial {
    uint32_t materialID;
    hg_vec4 albedo;
    hg_vec4 specularAlbedo;
    float metallic;
    float roughness;
    hg_vec4 emissive;
    PackedRayMedium rayMedium;
} PackedHalogenMaterial;

/* HalogenTriangle, RP:57-66 (72 B) */
typedef struct HalogenTriangle {
    hg_vec3 pointA, pointB, pointC;
    hg_vec3 normalA, normalB, normalC;
} HalogenTriangle;

/* BVHEntry, RP:68-76 (32 B).  triangleCount > 0: leaf, indexA = first triangle (mesh-relative);
 * triangleCount == 0: inner node, children at indexA and indexA+1 (mesh-relative node indices). */
typedef struct BVHEntry {
    uint32_t indexA;
    uint32_t triangleCount;
    hg_vec3 boundingCornerA;
    hg_vec3 boundingCornerB;
} BVHEntry;

/* ----------------------------------------------------------------------------------------------
 * Uniform block: every shader uniform of HalgoenCompute.compute:26-68,185, as set by
 * DispatchHalogenTrace (RP:359-401).  Field order is ours; meanings are the reference's.
 * -------------------------------------------------------------------------------------------- */
typedef struct hg_params {
    hg_mat4 camLocalToWorld;        /* CamLocalToWorldMatrix = camera.transform.localToWorldMatrix (RP:366) */
    hg_vec4 screenParameters;       /* (pixelWidth, pixelHeight, 0, 0) (RP:367) */
    hg_vec4 viewParameters;         /* (w, h, near, far) with h = tan(fov/2)*near, w = aspect*h (RP:361-368) */
    hg_vec4 cameraParameters;       /* camera position (RP:369) — dead in the kernel, kept for fidelity */
    int32_t frameCount;             /* FrameCount of the FIRST frame hg_render traces (RP:378) */
    uint32_t samplesPerPixel;       /* RP:382 */
    uint32_t maxBounces;            /* RP:383 */
    uint32_t maxDiffuseBounces;     /* RP:384 */
    uint32_t maxGlossyBounces;      /* RP:385 */
    uint32_t maxTransmissionBounces;/* RP:386 */
    uint32_t halogenDebugMode;      /* 0 none, 1 albedo, 2 normal, 3 tri tests, 4 box tests, 5 combined (RP:389) */
    uint32_t triangleDebugDisplayRange; /* RP:390 */
    uint32_t boxDebugDisplayRange;  /* RP:391 */
    int32_t defaultHDRIMipLevel;    /* RP:379 */
    float focalPlaneDistance;       /* RP:393 */
    float focalConeAngle;           /* aperture angle in degrees (RP:394) */
    float filterRadius;             /* pixels (RP:395) */
    int32_t useEnvironmentCubemap;  /* RP:398 */
    hg_vec4 bufferCounts;           /* (spheres, meshes, 0, 0) (RP:381) */
} hg_params;

/* Work / traffic counters, summed over every traced path since the last hg_reset_counters.
 * tri_tests / aabb_tests are the reference's TriangleTests / AABBTests (HalgoenCompute.compute:412,428). */
typedef struct hg_counters {
    uint64_t paths;        /* pixel-samples traced (W*H*SPP per frame) */
    uint64_t rays;         /* get_ray_intersection calls (bounce iterations reaching :895) */
    uint64_t tri_tests;    /* triangle_intersection_doublesided calls */
    uint64_t aabb_tests;   /* ray_AABB_test calls inside BLAS traversal (2 per inner node visit) */
    uint64_t mesh_visits;  /* rays x meshes (world->local transforms) */
    uint64_t sphere_tests; /* rays x spheres (sphere AABB prefilters) */
    uint64_t hits;         /* accepted hits (hit.rayT < far) */
    double kernel_ms;      /* summed device time of whole hg_render dispatches (HIP events on the context stream) */
    uint64_t launches;     /* hg_render dispatches timed in kernel_ms */
    double trace_ms;       /* summed device time of the traversal kernel alone (only with HG_OPT_TIMING on) */
    uint64_t trace_launches; /* traversal kernel launches timed in trace_ms */
    uint64_t node_rounds;  /* megakernels: wave-level iterations of the BVH descent loop (SIMD utilisation of the
                              descent = aabb_tests / 2 / (64 * node_rounds)) */
    uint64_t tri_rounds;   /* megakernels: wave-level iterations of the leaf loop (tri_tests / (64 * tri_rounds)) */
    uint64_t last_kernel;  /* HG_KERNEL_* variant the last hg_render ran (AUTO resolved; debug views: MEGA) */
    uint64_t trace_cycles; /* regenerating / streaming megakernels: wave clock cycles (s_memtime) spent in BVH
                              traversal, summed over waves */
    uint64_t shade_cycles; /* ... and in the rest of the bounce (shading, sampling, ray generation, accumulation) */
    uint64_t shade_detail[4]; /* analysis builds (HG_PHASE_DETAIL=1) only, streaming kernel: wave clock cycles of
                                 hit resolve / material + BSDF / path end + camera ray / next-ray setup; else 0 */
    uint64_t shade_rounds; /* regenerating / streaming megakernels: wave-level iterations of the shading code (SIMD
                              utilisation of shading = rays / (64 * shade_rounds)) */
    uint64_t primary_misses; /* paths whose camera ray hits nothing (trace_ray's first iteration takes the miss branch,
                                HC:941): a one-ray path; primary_misses / paths is the share of near-free paths */
    uint64_t exec_fallbacks; /* HG_CHECK_EXEC builds only (hg_selftest HG_SELFTEST_BUILD): lane-events where the
                                distributed leaf test found a lane of its wave inactive and took the sequential leaf
                                loop; must stay 0 (its DPP scans need a full wave).  0 in product builds */
    double trace_busy_ms;  /* the union of the traversal kernel's timed launch intervals (HG_OPT_TIMING): launches on the
                              two trace streams overlap, so trace_ms counts shared time twice; trace_busy_ms /
                              trace_launches is the kernel's device time per launch */
    uint64_t order_faults; /* HG_CHECK_EXEC builds only: cost-order sorts whose output was not a permutation of the tiles
                              (a placement out of range, or a tile placed other than once), and words of a sort's
                              scratch or a queue launch's heads found non-zero when the next use starts; must stay 0.
                              0 in product builds */
    uint64_t scene_uploads;         /* hg_upload_scene calls that (re)built the device scene, since hg_create */
    uint64_t scene_uploads_skipped; /* ... and calls whose five arrays equalled the last upload's byte for byte, which
                                       change nothing and return at once (the reference re-uploads on every camera
                                       move: ClearAccumulation sets ObjectBuffersDirty, RP:262-268, 296-299) */
    uint64_t scene_uploads_partial; /* ... of scene_uploads, those whose triangles and BVH entries equalled the last
                                       upload's (objects moved, materials changed): only the mesh table, spheres and
                                       materials were rebuilt */
    uint64_t scene_uploads_vouched; /* ... of the skipped and partial ones, those whose triangles and BVH entries were
                                       vouched for by an unchanged geometry generation (hg_upload_scene_gen), not compared */
    uint64_t server_launches;       /* render server lifetimes started (HG_OPT_SERVER), since hg_create */
    uint64_t server_frames;         /* frames posted to a render server, since hg_create */
    uint64_t server_refused;        /* posts that met a closing render server (its close handshake had not read them),
                                       re-posted to a new lifetime; since hg_create */
    uint64_t frames_lost;           /* render server frames whose gate gave up (never 0 on a healthy device: each makes
                                       the accumulation invalid, HG_E_FRAME_LOST), since hg_create */
    uint64_t server_ahead;          /* frames a render server posted ahead of the host's calls (HG_OPT_SERVER_AHEAD),
                                       since hg_create */
} hg_counters;

typedef struct hg_ctx hg_ctx;

enum {
    HG_OK = 0,
    HG_E_INVALID = -1,   /* bad argument / state */
    HG_E_HIP = -2,       /* HIP runtime error (text from hipGetErrorString) */
    HG_E_NOMEM = -3,
    HG_E_NOSCENE = -4,
    HG_E_NOTARGET = -5,  /* hg_resize not called */
    HG_E_UNSUPPORTED = -6,
    HG_E_COMM = -7,      /* RCCL error (text from ncclGetErrorString) or a mismatched communicator */
    HG_E_FRAME_LOST = -8 /* a render server frame never completed (HG_OPT_SERVER): its blend and every later one were
                            skipped, and the accumulation is invalid until hg_clear_accumulation / hg_set_accumulation
                            (hg_render refuses; the readbacks still hand out the accumulation through the last frame
                            blended, and return this code) */
};

/* Kernel variants selectable with hg_set_option(ctx, HG_OPT_KERNEL, v); all produce bit-identical images.
 * MEGA_REGEN: one lane per pixel of an 8x8-tile wave, one bounce per loop iteration; a lane whose path
 *   ends starts its next sample / frame at once (per-lane path regeneration), so no lane idles until the
 *   longest path of its wave ends.  Falls back to MEGA when maxBounces > 250 or samplesPerPixel >= 65535.
 * MEGA: the lockstep form — each lane traces whole paths, frame after frame (also runs the debug views 1-5).
 * MEGA_STREAM: MEGA_REGEN with a resumable traversal — lanes that finished traversing shade and start their next
 *   ray while the stragglers keep traversing (same limits and fallback as MEGA_REGEN).
 * AUTO (default): MEGA_STREAM when the scene has a BLAS deeper than 16 levels or at least 4 meshes, else MEGA_REGEN.
 * WAVEFRONT and MEGA_POOL (gen/trace/shade kernels over compacted ray queues; several tiles' paths per wave) were
 *   measured slower, rejected, and removed in round 5: selecting them returns HG_E_UNSUPPORTED. */
enum { HG_KERNEL_MEGA = 0, HG_KERNEL_WAVEFRONT = 1, HG_KERNEL_MEGA_REGEN = 2, HG_KERNEL_MEGA_STREAM = 3,
       HG_KERNEL_MEGA_POOL = 4, HG_KERNEL_AUTO = 5 };
/* HG_OPT_BLOCK: workgroup size of the lockstep kernel HG_KERNEL_MEGA (64/128/256; the debug views, large-maxBounces
 *   fallback); the regenerating / streaming kernels always run one-wave workgroups (their per-lane LDS rows assume it) and ignore it.  HG_OPT_COUNTERS: work counters on/off.
 * HG_OPT_TIMING: time every traversal-kernel launch with HIP events (hg_counters.trace_ms).
 * HG_OPT_REFILL: (the removed wavefront pipeline's dequeue threshold) returns HG_E_UNSUPPORTED.
 * HG_OPT_FRAME_SPLIT: regenerating kernel, waves per tile that trace disjoint frame ranges (their colours are then
 *   blended in frame order, bit-identical): 0 = automatic (about 6 launches' worth of the GPU's wave slots per
 *   launch — keeps small images and one rank's 1/N share at N GPUs filling the GPU), 1 = never, k = k per tile.
 * HG_OPT_DESCENT_T: traversal descent loop, leave it once at most this many lanes are still descending (the others
 *   test their leaves meanwhile; each lane's own step order is unchanged): -1 = automatic (for BLAS deeper than 16
 *   levels 3, or 8 with the streaming kernel; else 0 = classic while-while), 0..64 = fixed.
 * HG_OPT_TILE_ORDER: regenerating / streaming kernels, 1 (default) = each launch dispatches its tiles by descending
 *   wave time in the previous launches (shorter drain tail; same image), 0 = tile-index order.
 * HG_OPT_COALESCE: hg_render is asynchronous, so consecutive calls (same parameters, same accumulate flag) are held and
 *   launched together once this many frames are pending (default 32), or as soon as any other entry point is called
 *   (each launches the held frames first).  The frames, their order and the image are those of separate launches; a
 *   launch has a fixed cost (its drain tail: ~0.35 ms on C3), so the reference's one call per frame (RP:327) runs at
 *   the multi-frame rate.  A rank's share of the image (hg_set_tiling, N > 1) holds at least until its launch fills the
 *   GPU as one context's launch of the whole image does (6 rounds of the wave slots in 64-frame tile waves, at most
 *   1024 frames: 8 calls of 64 frames for a 1/8 share of 1080p).  1 = every call launches at once. */
/* HG_OPT_READBACK_DEPTH: display readbacks (hg_readback_begin[_format]) that may be outstanding at once, 1..16
 *   (default 2: display one frame behind).  A deeper ring lets a caller that displays every frame keep more frames in
 *   flight (display latency traded for throughput); changing it needs no readback outstanding. */
enum { HG_OPT_KERNEL = 1, HG_OPT_BLOCK = 2, HG_OPT_COUNTERS = 3, HG_OPT_TIMING = 4, HG_OPT_REFILL = 5,
       HG_OPT_FRAME_SPLIT = 6, HG_OPT_DESCENT_T = 7, HG_OPT_TILE_ORDER = 8, HG_OPT_COALESCE = 9,
       HG_OPT_READBACK_DEPTH = 10, HG_OPT_READBACK_STREAM = 11, HG_OPT_WAVE_UNITS = 12,
       HG_OPT_LANE_PICK = 14, HG_OPT_SERVER = 15, HG_OPT_SERVER_IDLE_US = 16, HG_OPT_SERVER_GATE_US = 17,
       HG_OPT_QUEUE_FILL = 18, HG_OPT_SERVER_AHEAD = 19 };
/* HG_OPT_SERVER_AHEAD (default 4): with the counters off (HG_OPT_COUNTERS 0), the render server traces this many frames
 *   ahead of the host's calls (the next frames of the same parameters and FrameCount chain), and serves a host that
 *   waits for every frame (a per-frame display) once two calls continue a chain.  A frame is blended only when the host
 *   asks for it, so the images are those of one launch per call; frames traced ahead and never asked for (the camera
 *   moved, the target was read, anything that stops the server) are abandoned, up to a unit per wave of them still
 *   traced.  0 = never.  (With the counters on, the counters would count frames never asked for: no tracing ahead.) */
/* HG_OPT_QUEUE_FILL (default 1): a streaming launch of more than 8 frames with fewer than this many rounds of the GPU's
 *   wave slots in 64-frame tile waves (tiles x frames / 64; a rank's 1/N share of the image at N GPUs launched a call at
 *   a time) runs the persistent work-queue form, its waves pulling (tile, frame chunk) units instead of one short wave
 *   per chunk.  0 = never.  Same images. */
/* HG_OPT_SERVER (default 1): hg_render calls of at most 8 accumulating frames on the streaming kernel (the reference's
 *   one dispatch per frame, RP:327) post their frames to a render server — persistent trace waves that outlive the call
 *   and take each posted frame's (tile, frame) units as soon as lanes free up, so one frame's last paths overlap the
 *   next frame's first — instead of launching.  Each frame's blend runs on the context stream behind a gate on that
 *   frame's completion, in frame order, so every readback / gather sees exactly the frames rendered before it.  The
 *   server is stopped (its waves trace what was posted, then leave) by uploads, resize, tiling, options, counters,
 *   hg_synchronize, hg_destroy, a launch of another kind, or parameters / FrameCount that do not continue its chain.
 *   1 (automatic) uses the server while the host runs ahead of the GPU (the call before last still in flight on the
 *   device: a host that queues frames), and, when it may trace ahead (HG_OPT_SERVER_AHEAD, counters off), once two
 *   calls continue a chain (a host that waits for each frame: a per-frame display); otherwise a call launches.
 *   2 = always (while the calls qualify).  0 = every call launches (the round-4 per-launch pipeline).  Same images
 *   either way.
 * HG_OPT_SERVER_IDLE_US (default 200000): a server with nothing new posted for this long closes itself (its waves
 *   leave the GPU).  Whether a post is taken never depends on a clock: one wave closes the server by a handshake with
 *   the host's post (both store, then load), and a post the closing wave did not see is re-posted to a new server
 *   (hg_counters.server_refused).  0..40000000; small values are for tests.
 * HG_OPT_SERVER_GATE_US (default -1: 30 s): a server frame whose gate waits this long is lost (HG_E_FRAME_LOST); a
 *   frame still short once every wave of its server has left is lost at once.  For tests and diagnostics. */
/* HG_OPT_READBACK_STREAM: 1 = each display readback is untiled into a device image of its own and copied to the host
 *   on a side stream, so the context stream (the next frames' blends) never waits for a copy; 0 = untiled into one
 *   device image and copied on the context stream; 2 = zero copy: the untile kernel writes the display image straight
 *   into the ring's pinned host image (mapped, fine-grained), no copy.  Same images either way. */
#define HG_READBACK_MAX 16
/* HG_OPT_WAVE_UNITS: streaming launches of more than 8 frames without a frame split, tiles traced per wave (1..4;
 *   0 = automatic, which is 1: more tiles per wave measured slower).  Images whose size is not
 *   a multiple of 8 always trace one tile per wave.  Same images and counters either way.
 * HG_OPT_LANE_PICK (default 1): launches of at most 8 frames go to the first trace stream whose previous trace and blend are done
 *   (1), or to the trace streams in turn (0).  Same images either way. */
int hg_abi_version(void);

/* Create a context on HIP device `device` (ordinal as seen by the process). */
int hg_create(int device, hg_ctx** out);
void hg_destroy(hg_ctx* ctx);
const char* hg_last_error(const hg_ctx* ctx);

/* Upload the scene buffers (UpdateObjectBuffers, RP:448-509).  Validates every cross-reference
 * (offsets, child indices, material indices) before anything reaches the GPU.  Arrays equal byte for byte to the last
 * successful upload's are detected (a parallel compare against retained host copies) and change nothing: the call
 * returns without touching the device (hg_counters.scene_uploads_skipped).  When only the spheres, the meshes'
 * matrices / materials or the materials changed (triangles, BVH entries and every mesh's buffer offsets as before),
 * only those tables are rebuilt (hg_counters.scene_uploads_partial). */
int hg_upload_scene(hg_ctx* ctx,
                    const HalogenSphere* spheres, int32_t n_spheres,
                    const HalogenMeshData* meshes, int32_t n_meshes,
                    const PackedHalogenMaterial* materials, int32_t n_materials,
                    const HalogenTriangle* triangles, int32_t n_triangles,
                    const BVHEntry* blas, int32_t n_nodes);
/* hg_upload_scene with the caller's geometry generation: a non-zero generation equal to the last successful upload's
 * vouches that the triangles and BVH entries are that upload's (the caller bumps it whenever its mesh registry —
 * RayTracingManager's mesh list in the reference — changes), so they are not compared; the spheres, mesh records and
 * materials are compared as always (the reference re-reads transforms and materials on every re-upload, RP:448-509).
 * The reference re-uploads every buffer on each camera move (RP:262-268, 296-299): this keeps that call pattern at the
 * cost of the small arrays only.  Generation 0 (and every generation change) compares everything, as hg_upload_scene;
 * an upload that compared everything adopts its generation for the next ones.  The vouch is trusted: triangles or BVH
 * entries changed in place under an unchanged generation (same counts) keep the device's previous geometry. */
int hg_upload_scene_gen(hg_ctx* ctx, uint64_t geometry_generation,
                        const HalogenSphere* spheres, int32_t n_spheres,
                        const HalogenMeshData* meshes, int32_t n_meshes,
                        const PackedHalogenMaterial* materials, int32_t n_materials,
                        const HalogenTriangle* triangles, int32_t n_triangles,
                        const BVHEntry* blas, int32_t n_nodes);

/* Environment cubemap (EnvironmentCubemap, HalgoenCompute.compute:48): RGBA32F texels, layout
 * [mip][face][y][x][4], faces +X,-X,+Y,-Y,+Z,-Z, mip m is max(1, face_size >> m) square.
 * Sampling is the manual bilinear defined in DESIGN.md §cubemap (shared with the oracle). */
int hg_upload_cubemap(hg_ctx* ctx, int32_t face_size, int32_t n_mips, const float* texels, size_t n_floats);

int hg_set_params(hg_ctx* ctx, const hg_params* params);

/* (Re)allocate the accumulation target for a width x height image and clear it (OnCameraSetup). */
int hg_resize(hg_ctx* ctx, int32_t width, int32_t height);

/* Multi-GPU: this context renders only the 8x8 tiles t with t % n_ranks == rank (tile-row-major order). */
int hg_set_tiling(hg_ctx* ctx, int32_t rank, int32_t n_ranks);

int hg_clear_accumulation(hg_ctx* ctx);

/* Trace n_frames consecutive frames, FrameCount = params.frameCount + k, each followed by the
 * progressive blend acc = acc*(1-w) + new*w with w = 1.0f/FrameCount (AccumulationShader.shader:33).
 * accumulate == 0 reproduces Accumulate=false: FrameCount forced to 1 and acc = new each frame.
 * Asynchronous on the context stream (the frames may be held for one launch with later calls: HG_OPT_COALESCE). */
int hg_render(hg_ctx* ctx, int32_t n_frames, int32_t accumulate);

int hg_synchronize(hg_ctx* ctx);

/* Row-major RGBA32F image (width*height*4 floats) of the accumulation target.  With tiling, only this
 * rank's pixels are written; the others are left untouched. Blocks. */
int hg_readback(hg_ctx* ctx, float* rgba, size_t n_floats);

/* Display readback, pipelined (the reference's per-frame Blit to rtCameraColor, RP:343-347, as a host image):
 * hg_readback_begin_format enqueues, after every frame rendered so far, the untiling of the accumulation target into a
 * row-major image in a display format and its copy into the next of the context's pinned host images (a ring of
 * HG_OPT_READBACK_DEPTH, default 2), and returns at once; hg_readback_end_data waits for the OLDEST begun readback and
 * hands out its image (with tiling, other ranks' pixels are 0).  At most HG_OPT_READBACK_DEPTH readbacks are
 * outstanding, so a caller can trace frame k+1 while frame k's image crosses PCIe:
 *   render(1); begin; if (depth outstanding) end -> display        (one frame behind at depth 2)
 * The pointer stays valid until the depth-th hg_readback_begin after the one it came from, or until hg_resize /
 * hg_set_tiling / hg_destroy.  hg_readback_end launches no held frames (the begin already did).
 * Formats (csrc/hg_pack.h has the exact conversion; the fp32 accumulation target is never changed):
 *   HG_DISPLAY_RGBA32F     16 B/px, the accumulation target as it is;
 *   HG_DISPLAY_RGBA16F      8 B/px, IEEE half per channel, round to nearest even, overflow to Inf, NaN -> 0x7E00;
 *   HG_DISPLAY_R11G11B10F   4 B/px, DXGI_FORMAT_R11G11B10_FLOAT (R bits 0-10, G 11-21, B 22-31, no alpha): the URP
 *                           HDR camera target the reference blits into (URP-HighFidelity.asset:26-27,
 *                           m_HDRColorBufferPrecision 0); round to nearest even, overflow to +Inf, negatives and NaN
 *                           to 0 (D3D's converter cannot run here: parity with it is unpinned).
 * hg_readback_begin / hg_readback_end are the RGBA32F forms (hg_readback_end refuses a readback of another format). */
enum { HG_DISPLAY_RGBA32F = 0, HG_DISPLAY_RGBA16F = 1, HG_DISPLAY_R11G11B10F = 2 };
int hg_readback_begin_format(hg_ctx* ctx, int32_t format);
int hg_readback_end_data(hg_ctx* ctx, const void** data, size_t* n_bytes, int32_t* format);
int hg_readback_begin(hg_ctx* ctx);
int hg_readback_end(hg_ctx* ctx, const float** rgba, size_t* n_floats);
/* The display packing on the host (no device work): n_pixels RGBA32F pixels into `out` (16 / 8 / 4 B per pixel), the
 * same conversion the device applies in hg_readback_begin_format. */
int hg_pack_display(const float* rgba, size_t n_pixels, int32_t format, void* out);

/* Checkpoint / resume: the inverse of hg_readback.  The reference's whole resumable state is the accumulation target
 * and FrameCount (RP:152, RP:185, RP:347).  Loads a row-major RGBA32F image (width*height*4 floats, as hg_readback
 * returns it; with tiling only this rank's pixels are read) into the accumulation target and sets the FrameCount the
 * next accumulated frame is traced with (frame_count >= 1; a later hg_set_params supplies its own frameCount).
 * readback -> new context -> hg_set_accumulation -> hg_render continues bit-identically.  Blocks. */
int hg_set_accumulation(hg_ctx* ctx, const float* rgba, size_t n_floats, int32_t frame_count);

/* Device-to-device copy of this rank's packed tiles (n_local_tiles * 64 * 4 floats, tile-major,
 * pixel (lx,ly) of a tile at lx + 8*ly) into caller-owned device memory on the same device.  Returns after the copy
 * has completed on the context stream; a consumer on another stream or engine must order itself after the call.
 * (The multi-GPU path uses hg_comm_gather instead, which stays on the contexts' own streams.) */
int hg_copy_tiles_device(hg_ctx* ctx, void* dst_device, size_t n_bytes);
int32_t hg_local_tile_count(const hg_ctx* ctx);

int hg_get_counters(const hg_ctx* ctx, hg_counters* out);
int hg_reset_counters(hg_ctx* ctx);

/* Tuning knobs (kernel variant, lockstep block size, counters on/off, ...: the HG_OPT_* above). */
int hg_set_option(hg_ctx* ctx, int32_t option, int32_t value);

/* Device self-tests of arithmetic shortcuts the kernels rely on (and the build's compiled-in checks).  HG_SELFTEST_RCP: the fast correctly-rounded
 * reciprocal against IEEE 1.0f/x for every float of its range.  Returns the number of mismatches (must be 0),
 * or a negative error; *tested (optional) receives the number of inputs checked. */
enum { HG_SELFTEST_RCP = 1, HG_SELFTEST_BUILD = 2 };
/* HG_SELFTEST_BUILD returns a bit mask of the run-time checks and A/B switches compiled into this build (no device
 * work): HG_BUILD_CHECK_EXEC, the run-time precondition checks (make check_exec); HG_BUILD_NO_REGEN_ITEMS, the
 * regenerating kernel without (pixel, frame) item scheduling (make noitems). */
enum { HG_BUILD_CHECK_EXEC = 1, HG_BUILD_NO_REGEN_ITEMS = 2 };
int64_t hg_selftest(hg_ctx* ctx, int32_t test, int64_t* tested);

/* ----------------------------------------------------------------------------------------------
 * Multi-GPU framebuffer gather (not in the reference, which is single-GPU).
 * Every rank renders the 8x8 tiles t % n_ranks == rank of the same image (hg_set_tiling) with its own context, on
 * its own GPU; the only exchange is one gather of the ranks' accumulated tiles to the root, which assembles the
 * row-major image on its device.  Two ways to build the communicator over the rank contexts:
 *   hg_comm_init_rank  one process per GPU (e.g. under torchrun, MPI, or any launcher): rank 0 makes an id with
 *                      hg_comm_unique_id, the caller distributes it, every rank joins (blocks until all have);
 *   hg_comm_init_all   one process driving all the contexts (e.g. the C# render pass with one context per GPU,
 *                      one host thread per device for hg_render): a single call over all contexts.
 * Transport: RCCL point-to-point over xGMI (ncclSend / ncclRecv on each context's own stream, so the gather is
 * ordered after that context's renders with no host wait).  hg_comm_init_all over contexts that share a device
 * (a one-GPU rehearsal; RCCL refuses two ranks on one GPU) uses in-process device copies instead, ordered by events.
 * The comm does not own the contexts; destroy it before them.  Not thread-safe.
 * -------------------------------------------------------------------------------------------- */
typedef struct hg_comm hg_comm;
#define HG_COMM_ID_BYTES 128   /* = NCCL_UNIQUE_ID_BYTES */
enum { HG_COMM_RCCL = 1, HG_COMM_PEER = 2 };

/* A fresh communicator id (ncclGetUniqueId): made once, by the root process, and handed to every rank. */
int hg_comm_unique_id(uint8_t id[HG_COMM_ID_BYTES]);
/* This process's rank of an n_ranks communicator; ctx must already be tiled as (rank, n_ranks). Blocks until every
 * rank has joined. */
int hg_comm_init_rank(hg_ctx* ctx, int32_t n_ranks, const uint8_t id[HG_COMM_ID_BYTES], int32_t rank,
                      hg_comm** out);
/* All ranks in this process: ctxs[r] is rank r of n_ranks (each already tiled as (r, n_ranks)). */
int hg_comm_init_all(hg_ctx* const* ctxs, int32_t n_ranks, hg_comm** out);
/* Collective (every rank calls it; with hg_comm_init_all one call covers all ranks): gather the ranks' accumulated
 * tiles to `root`, which assembles the full row-major RGBA32F image on its device.  Asynchronous on the contexts'
 * streams.  All ranks must have the same target size. */
int hg_comm_gather(hg_comm* comm, int32_t root);
/* Wait until this process's ranks have finished the last gather (sends done; on the root, image assembled).  Like every
 * wait of hg_comm it is bounded: RCCL errors (ncclCommGetAsyncError) and a deadline that starts once this process's own
 * renders have retired end it with HG_E_COMM and abort the communicator (a dead or stalled peer never hangs the caller).
 * A failed agreement (ranks with different target sizes or tilings) fails hg_comm_gather on every rank alike. */
int hg_comm_synchronize(hg_comm* comm);
/* On the process holding the root (after hg_comm_gather): the assembled image, width*height*4 floats. Blocks, with the
 * deadline of hg_comm_synchronize. */
int hg_comm_readback(hg_comm* comm, float* rgba, size_t n_floats);
/* Pipelined display of the gathered image (the multi-GPU form of hg_readback_begin_format / hg_readback_end_data; same
 * formats): begin enqueues, after the last hg_comm_gather, the conversion of the root's assembled image and its copy
 * into the root context's ring of pinned host images (that context's HG_OPT_READBACK_DEPTH) and returns at once; end
 * waits for the oldest begun one with the deadline of hg_comm_synchronize and hands out its image. */
int hg_comm_readback_begin(hg_comm* comm, int32_t format);
int hg_comm_readback_end(hg_comm* comm, const void** data, size_t* n_bytes, int32_t* format);
/* The deadline of every wait (default 120000 ms, or the environment variable HALOGEN_COMM_TIMEOUT_MS at init). */
int hg_comm_set_timeout_ms(hg_comm* comm, int64_t timeout_ms);
int hg_comm_transport(const hg_comm* comm);     /* HG_COMM_RCCL or HG_COMM_PEER */
const char* hg_comm_last_error(const hg_comm* comm);
void hg_comm_destroy(hg_comm* comm);
/* Host twin of the root's assembly (no device work): slabs = [n_ranks][slab_tiles][64] RGBA32F tiles, slab r holding
 * rank r's accumulated tiles in its local order (as hg_copy_tiles_device packs them); writes the row-major
 * width*height*4 image.  Shares the tile -> rank / slot / pixel mapping with the device assembly (csrc/hg_tiling.h). */
int hg_comm_assemble_host(const float* slabs, int64_t slab_tiles, int32_t width, int32_t height, int32_t n_ranks,
                          float* rgba, size_t n_floats);

/* ----------------------------------------------------------------------------------------------
 * Host-side data producers (the reference keeps these in C#: BVHGenerator.cs, RayTracingMesh.cs,
 * HalogenRenderPass.UpdateObjectBuffers).  Restated in C++ with the reference's float semantics,
 * so a non-Unity caller can build the buffers hg_upload_scene takes.
 * -------------------------------------------------------------------------------------------- */

/* BVHGenerator.GenerateMeshBVH (BVHGenerator.cs:13-134).  `indices` (3*n_tris) is REORDERED IN PLACE,
 * exactly as the reference reorders its triangle list.  root_min/root_max = Unity mesh.bounds.min/max.
 * Writes at most max_nodes entries; returns the node count (or a negative error / the required count
 * negated-minus-one if max_nodes is too small). */
int64_t hg_build_blas(const float* vertices, int32_t n_vertices, int32_t* indices, int32_t n_tris,
                      const float root_min[3], const float root_max[3], int32_t max_hierarchy_depth,
                      BVHEntry* out_nodes, int64_t max_nodes);

/* hg_build_blas with n_threads workers (0: all hardware threads): the same node array and the same reordered
 * `indices` (tests/test_bvh.py), level-parallel over the BFS queue and rank-parallel inside large nodes. A vertex
 * array holding a NaN, or fewer than 4096 triangles, takes the sequential build. */
int64_t hg_build_blas_mt(const float* vertices, int32_t n_vertices, int32_t* indices, int32_t n_tris,
                         const float root_min[3], const float root_max[3], int32_t max_hierarchy_depth,
                         BVHEntry* out_nodes, int64_t max_nodes, int32_t n_threads);

/* Fast BLAS, NOT the reference's hierarchy (an SAH variant behind a non-parity choice): a
 * binned surface-area-heuristic build into the same BVHEntry format (children of g at indexA, indexA + 1; leaves of at
 * most max_leaf <= 15 triangles, ranges of the reordered `indices`; min/max boxes through the reference's Bounds
 * arithmetic, padded when thin as BVHGenerator pads them; depth < max_depth).
 * Any caller may pass its nodes to hg_upload_scene in place of hg_build_blas's: the render is then a different valid
 * hierarchy's (the same nearest triangles except within rounding, other traversal counters).  Returns the node count,
 * -(count + 1) if max_nodes is too small, or HG_E_INVALID / HG_E_UNSUPPORTED (the depth cap left a leaf over 15). */
int64_t hg_build_blas_sah(const float* vertices, int32_t n_vertices, int32_t* indices, int32_t n_tris,
                          int32_t max_leaf, int32_t max_depth, BVHEntry* out_nodes, int64_t max_nodes);

/* Unity Bounds.SetMinMax(min,max) followed by .min/.max (centre/extents round trip) — the arithmetic
 * every bound in the reference goes through (BVHGenerator.cs:171-183, RayTracingMesh.cs:106-117). */
void hg_unity_bounds(const float in_min[3], const float in_max[3], int32_t pad_if_thin,
                     float out_min[3], float out_max[3]);

/* RayTracingMesh.UpdateTriangleList (RayTracingMesh.cs:70-87). */
int hg_pack_triangles(const float* vertices, const float* normals, int32_t n_vertices,
                      const int32_t* indices, int32_t n_tris, HalogenTriangle* out);

#ifdef __cplusplus
}
#endif
#endif /* HALOGEN_ABI_H */
