// hg_ctx.h — the context object behind the C-ABI's opaque hg_ctx (private to libhalogen_hip.so; shared by
// hg_runtime.hip and hg_comm.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "halogen_abi.h"
#include "hg_layout.h"

struct DevBuf {  // a device allocation owned by a context
    void* p = nullptr;
    size_t bytes = 0;
};

struct hg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // scene
    bool has_scene = false;
    DevBuf spheres, meshes, materials, nodes, leaves, tris, normals;
    int32_t n_spheres = 0, n_meshes = 0, n_materials = 0, n_tris = 0, n_nodes = 0;
    uint32_t stack_depth = 2;
    // the caller's arrays of the last upload (spheres, meshes, materials, triangles, BVH entries), byte for byte: an
    // identical re-upload (the reference re-uploads on every camera move) is detected and skipped
    std::vector<uint8_t> scene_copy[5];
    std::vector<HgDevMesh> dev_meshes;  // the device mesh table of the last upload (partial re-uploads start from it)
    uint64_t scene_uploads = 0, scene_uploads_skipped = 0, scene_uploads_partial = 0, scene_uploads_vouched = 0;
    uint64_t geometry_gen = 0;  // hg_upload_scene_gen: the caller's geometry generation of the last upload (0: none)

    // cubemap
    DevBuf cube;
    int32_t cube_size = 0, cube_mips = 0;
    uint32_t cube_mip_offset[HG_MAX_CUBE_MIPS] = {};

    // params
    bool has_params = false;
    hg_params params{};

    // target
    int32_t W = 0, H = 0, rank = 0, n_ranks = 1, tiles_x = 0, tiles_y = 0, n_local_tiles = 0;
    DevBuf acc;

    DevBuf spill;  // traversal stack entries beyond the LDS part, per thread, of launches on the context stream
    // Trace pipeline (hg_render): the regenerating / streaming kernels trace each launch chunk on one of HG_TRACE_LANES
    // side streams, in turn, into that stream's own frame-colour buffer; the chunk's in-order blend into the accumulator
    // runs on `stream`.  So a chunk's tail overlaps the next chunk's trace, and everything else on `stream` (readback,
    // clear, gather) stays ordered after the blends.  Per trace stream: its buffers and the events that order them.
    struct TraceLane {
        hipStream_t stream = nullptr;
        hipEvent_t traced = nullptr;   // after this stream's last trace (the blend on `stream` waits for it)
        hipEvent_t blended = nullptr;  // after the blend of this stream's last chunk (its buffers are free again)
        bool blend_pending = false;    // `blended` was recorded and the next trace here must wait for it
        DevBuf frame_color;            // this chunk's per-frame colours ([slot][frame], fc_index)
        DevBuf spill;                  // traversal stack entries beyond the LDS part, one column per thread
        // Cost order: this stream's traces add their wave times to tile_cost and its sorts read and clear them, all in
        // this stream's order.  (One buffer shared by both streams let a sort read costs that the other stream's trace
        // was still adding to: the counting sort's two passes then disagreed and wrote out of range.)
        DevBuf tile_cost;              // per local tile, wave-clock cost since this stream's last sort
        DevBuf tile_order;             // the cost order this stream's launches read
        DevBuf order_scratch;          // hg_order_tiles: histogram and claims (zeroed at allocation, left zeroed)
        DevBuf queue;                  // kQueue launches: the 8 unit heads + exit count (zeroed at allocation; the
                                       // last wave of each launch zeroes them again)
        bool tile_cost_valid = false;  // tile_cost holds costs for this tiling
        bool tile_order_valid = false;
        int64_t frames_since_order = 0;  // frames traced on this stream since its last sort
    };
    static_assert(HG_TRACE_LANES_BIG >= 1 && HG_TRACE_LANES_BIG <= HG_TRACE_LANES, "HG_TRACE_LANES_BIG out of range");
    TraceLane lanes[HG_TRACE_LANES];
    int next_lane = 0;     // chunks of at most HG_QUEUE_MAX_FRAMES frames: every lane in turn
    int next_lane_big = 0;  // longer chunks: lanes [0, HG_TRACE_LANES_BIG) in turn

    // The render server (hg_mega.hip kServer): launches of the reference's one frame per call
    // (at most HG_QUEUE_MAX_FRAMES frames, accumulating, streaming kernel) post their frames to persistent trace waves
    // that outlive the call, instead of launching; each frame's blend runs on `stream` behind a gate on its completion
    // count.  Stopped (the waves drain what was posted and leave) by every entry point that changes what the waves
    // read, by another kind of launch, and when its parameters or FrameCount chain do not continue.
    struct Server {
        hipStream_t stream = nullptr;  // CU-masked: a hardware queue of its own (never ahead of `stream`'s gates)
        bool running = false;
        DevBuf ctl;         // heads, mirror, ticket (HG_SV_CTL_BYTES), zeroed before each launch
        DevBuf done;        // per ring slot a completion count on its own 128-B line, zeroed before each launch
        DevBuf ring;        // colour ring: ring_n frames of n_local_tiles * 64 float4
        DevBuf spill, tile_cost, tile_order, order_scratch;
        bool tile_cost_valid = false;
        unsigned long long* host = nullptr;  // pinned, coherent: the host words HG_SV_HOST_* (hg_layout.h)
        uint32_t ring_n = 0, posted = 0, cap = 0;
        uint32_t committed = 0;  // frames the host asked for (gate + blend queued); posted - committed were posted ahead
        uint32_t uses[HG_SV_RING] = {};     // frames posted to each ring slot in this lifetime
        hipEvent_t blended[HG_SV_RING] = {};  // after the blend of each ring slot's last frame
        // HALOGEN_SERVER_SERIAL=1 (a profiling aid, tools/pmc_server.sh): the gates wait for the lifetime's end (this
        // event, after the server kernel), so a profiler that runs one kernel at a time (rocprofv3 --pmc) never runs a
        // gate before the server it waits for
        hipEvent_t exited = nullptr;
        bool blend_valid[HG_SV_RING] = {};
        hg_params params{};   // the parameters it was started with (frameCount: its first frame)
        int32_t kernel_variant = 0, descent_t = 0;
        HgKernelParams kp{};  // the launch's parameters (the blends read acc / ring / first_frame)
        int32_t idle_us = HG_SV_IDLE_US;  // HG_OPT_SERVER_IDLE_US
        int64_t gate_us = -1;             // HG_OPT_SERVER_GATE_US (< 0: the default, 30 s)
#if HG_SV_DIAG_TIMES
        double post_s[256] = {};  // (analysis builds) host clock of each post
#endif
    } sv;
    int32_t server_on = 1;  // HG_OPT_SERVER
    uint64_t server_launches = 0, server_frames = 0;
    uint64_t server_refused = 0;  // posts that met a closing server (the close handshake), re-posted to a new one
    // HG_OPT_SERVER_AHEAD: frames the server traces ahead of the host's calls (counters off), and the call chain that
    // engages the server without a host running ahead: consecutive accumulating calls with the same parameters, each
    // continuing the last one's FrameCount
    int32_t sv_ahead = HG_SV_AHEAD;
    uint64_t server_ahead_posts = 0;
    hg_params chain_params{};
    int32_t chain_next = 0, chain_len = 0;
    // Lost frames (a server frame's gate gave up, hg_server_gate): the gate raises `lost` (uncached device memory), and
    // every later blend into the accumulator is skipped; the host marks the accumulator invalid (acc_lost) when it reads
    // the gate's host word and the frame belongs to the current accumulation (acc_epoch: advanced by every clear,
    // checkpoint load and reallocation, which also reset both).  While acc_lost, hg_render and every readback / copy /
    // gather of the accumulator return HG_E_FRAME_LOST.
    DevBuf lost;
    uint32_t acc_epoch = 0;
    bool acc_lost = false;
    uint64_t frames_lost = 0;
    // The server serves only a host that runs ahead: each render call records call_done[calls & 1] on `stream` after
    // its frames' blends, so at a call the event of the call before last tells whether the GPU still works on it
    hipEvent_t call_done[2] = {};
    bool call_done_valid[2] = {};
    uint64_t calls = 0;

    // counters / timing
    DevBuf counters_dev;
    hg_counters counters{};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending, free_events, pending_trace;

    // device / options
    int n_cu = 0;
    int32_t kernel = HG_KERNEL_AUTO, block = 128, counters_on = 1, timing = 0;
    int32_t frame_split = 0;  // 0: automatic (see hg_render)
    int32_t wave_units = 0;   // HG_OPT_WAVE_UNITS, 0: automatic (see hg_render)
    int32_t lane_pick = HG_LANE_PICK;  // HG_OPT_LANE_PICK: 1-frame chunks on the first idle trace stream (1) or in turn (0)
    int32_t descent_t = -1;   // < 0: automatic from the BLAS depth
    int32_t tile_order_on = HG_TILE_ORDER;  // HG_OPT_TILE_ORDER
    int32_t queue_fill = HG_QUEUE_FILL;     // HG_OPT_QUEUE_FILL
    // Render coalescing (HG_OPT_COALESCE): hg_render is asynchronous, so consecutive calls with the same parameters are
    // held and launched as one multi-frame launch once `coalesce` frames are pending, or as soon as anything reads or
    // changes the context's state (every other entry point flushes first: hg_ctx_flush).  Same frames, same order,
    // same image; 1 = every call launches at once.
    int32_t coalesce = HG_COALESCE;
    int32_t pending_frames = 0, pending_acc = 0;

    // Display readback (hg_readback, hg_readback_begin[_format] / _end[_data]): the accumulator untiled on the device
    // into `image` (row-major, in the display format), then copied into the next of rb_depth pinned host images (a ring)
    DevBuf image;
    void* image_host[HG_READBACK_MAX] = {};
    size_t image_host_cap[HG_READBACK_MAX] = {};    // allocated bytes
    size_t image_host_bytes[HG_READBACK_MAX] = {};  // bytes of the readback it holds
    int32_t image_host_format[HG_READBACK_MAX] = {};
    bool image_host_mapped[HG_READBACK_MAX] = {};  // allocated mapped + fine-grained (HG_OPT_READBACK_STREAM 2)
    hipEvent_t image_copied[HG_READBACK_MAX] = {};
    int rb_depth = 2;                 // HG_OPT_READBACK_DEPTH: readbacks that may be outstanding
    int rb_side = HG_READBACK_SIDE;   // HG_OPT_READBACK_STREAM: copies on rb_stream from per-slot device images
    hipStream_t rb_stream = nullptr;
    DevBuf rb_image[HG_READBACK_MAX];
    hipEvent_t rb_untiled[HG_READBACK_MAX] = {};
    int rb_next = 0, rb_pending = 0;  // host image the next begin fills; begun readbacks not yet ended (<= rb_depth)
};

// Launch the held frames of a context, if any (hg_runtime.hip; every entry point but hg_render calls it first)
int hg_ctx_flush(hg_ctx* c);
// The context's accumulation is invalid (a render server frame was lost; reads the gates' report first)
bool hg_ctx_lost(hg_ctx* c);
// Enqueue a display readback (hg_readback_begin_format) from the accumulator (rows == nullptr) or from a row-major
// float4 image of the target's size on the context's device; and the copy event of the oldest outstanding one
int hg_ctx_display_begin(hg_ctx* c, const void* rows, int32_t format);
hipEvent_t hg_ctx_display_oldest(const hg_ctx* c);
