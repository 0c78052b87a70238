// hg_runtime.hip — implementation of the C-ABI in include/halogen_abi.h (context, uploads, dispatch,
// readback, counters).  Stands in for the ComputeBuffer / RTHandle / DispatchCompute / Blit calls of
// Assets/Scripts/Render Features/HalogenRenderPass.cs (RP:237-508).
//
// Error model: every entry point returns HG_OK or a negative HG_E_* code and never aborts; the text of
// the last error is kept per context (hg_last_error).  There is no CPU fallback: a missing GPU or a HIP
// failure is an error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "halogen_abi.h"
#include "hg_fmath.h"
#include "hg_layout.h"
#include "hg_ctx.h"
#include "hg_tiling.h"
#include "hg_interval.h"
#include "hg_pack.h"
#include "hg_host_pool.h"

hipError_t hg_launch_mega(const HgKernelParams& kp, int block, bool counters, hipStream_t stream);
hipError_t hg_launch_mega_regen(const HgKernelParams& kp, int block, bool counters, hipStream_t stream);
hipError_t hg_launch_mega_stream(const HgKernelParams& kp, int block, bool counters, hipStream_t stream,
                                 bool server = false);
hipError_t hg_launch_server_frame(float4* acc, const float4* colors, uint32_t n_slots, int32_t frame_count,
                                  const uint32_t* done, uint32_t target, uint64_t timeout_ticks,
                                  const unsigned long long* exitw, uint32_t* lost, unsigned long long* err,
                                  uint32_t epoch, hipStream_t stream);
hipError_t hg_launch_blend_frames(const HgKernelParams& kp, const uint32_t* lost, hipStream_t stream);
hipError_t hg_launch_order_tiles(unsigned long long* cost, uint32_t* order, uint32_t n, void* scratch,
                                 unsigned long long* faults, hipStream_t stream);
size_t hg_order_scratch_bytes(uint32_t n);
int64_t hg_selftest_rcp_all(int64_t* tested);

namespace {

constexpr size_t kFrameColorCap = size_t(4) << 30;  // frame-parallel colour buffer cap (bytes)
constexpr uint32_t kMaxStack = 64;  // LDS stack entries per lane; BLAS depth must be <= kMaxStack - 2
constexpr int kHostThreads = 16;    // host threads of hg_upload_scene's compare / repack (the GPU box's CPU share)

}  // namespace

namespace {

int fail(hg_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define HG_HIP(ctx, call)                                                                              \
    do {                                                                                               \
        hipError_t e_ = (call);                                                                        \
        if (e_ != hipSuccess) return fail((ctx), HG_E_HIP, "%s failed: %s", #call, hipGetErrorString(e_)); \
    } while (0)

int set_device(hg_ctx* c) {
    HG_HIP(c, hipSetDevice(c->device));
    return HG_OK;
}

void release(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

int upload(hg_ctx* c, DevBuf& b, const void* src, size_t bytes) {
    size_t alloc = std::max<size_t>(bytes, 16);  // the reference allocates >= 1 element (RP:544)
    if (b.bytes != alloc) {
        release(b);
        hipError_t e = hipMalloc(&b.p, alloc);
        if (e != hipSuccess) return fail(c, HG_E_NOMEM, "hipMalloc(%zu) failed: %s", alloc, hipGetErrorString(e));
        b.bytes = alloc;
    }
    if (bytes) HG_HIP(c, hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, c->stream));
    return HG_OK;
}

float4 f4(float x, float y, float z, float w) { return make_float4(x, y, z, w); }
float bits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
float bits(int32_t i) { float f; std::memcpy(&f, &i, 4); return f; }

// Padded world-space boxes of a mesh root's two children (for the exact mesh skip, hg_device.h mesh_live_mask).
// The local box corners go through the double-precision inverse of the float worldToLocal the kernel uses;
// the pad (1e-3 of the box size + 1e-4 of the coordinate magnitude + 1e-5) exceeds by orders of magnitude
// the float rounding of the reference's local-space slab test (~1e-7 relative), so "misses the padded box"
// implies "the reference's ray_AABB_test returns INF (or a tEntry beyond the closest hit)".
bool invert4(const double a[16], double out[16]) {
    double inv[16];
    inv[0] = a[5] * a[10] * a[15] - a[5] * a[11] * a[14] - a[9] * a[6] * a[15] + a[9] * a[7] * a[14] +
             a[13] * a[6] * a[11] - a[13] * a[7] * a[10];
    inv[4] = -a[4] * a[10] * a[15] + a[4] * a[11] * a[14] + a[8] * a[6] * a[15] - a[8] * a[7] * a[14] -
             a[12] * a[6] * a[11] + a[12] * a[7] * a[10];
    inv[8] = a[4] * a[9] * a[15] - a[4] * a[11] * a[13] - a[8] * a[5] * a[15] + a[8] * a[7] * a[13] +
             a[12] * a[5] * a[11] - a[12] * a[7] * a[9];
    inv[12] = -a[4] * a[9] * a[14] + a[4] * a[10] * a[13] + a[8] * a[5] * a[14] - a[8] * a[6] * a[13] -
              a[12] * a[5] * a[10] + a[12] * a[6] * a[9];
    inv[1] = -a[1] * a[10] * a[15] + a[1] * a[11] * a[14] + a[9] * a[2] * a[15] - a[9] * a[3] * a[14] -
             a[13] * a[2] * a[11] + a[13] * a[3] * a[10];
    inv[5] = a[0] * a[10] * a[15] - a[0] * a[11] * a[14] - a[8] * a[2] * a[15] + a[8] * a[3] * a[14] +
             a[12] * a[2] * a[11] - a[12] * a[3] * a[10];
    inv[9] = -a[0] * a[9] * a[15] + a[0] * a[11] * a[13] + a[8] * a[1] * a[15] - a[8] * a[3] * a[13] -
             a[12] * a[1] * a[11] + a[12] * a[3] * a[9];
    inv[13] = a[0] * a[9] * a[14] - a[0] * a[10] * a[13] - a[8] * a[1] * a[14] + a[8] * a[2] * a[13] +
              a[12] * a[1] * a[10] - a[12] * a[2] * a[9];
    inv[2] = a[1] * a[6] * a[15] - a[1] * a[7] * a[14] - a[5] * a[2] * a[15] + a[5] * a[3] * a[14] +
             a[13] * a[2] * a[7] - a[13] * a[3] * a[6];
    inv[6] = -a[0] * a[6] * a[15] + a[0] * a[7] * a[14] + a[4] * a[2] * a[15] - a[4] * a[3] * a[14] -
             a[12] * a[2] * a[7] + a[12] * a[3] * a[6];
    inv[10] = a[0] * a[5] * a[15] - a[0] * a[7] * a[13] - a[4] * a[1] * a[15] + a[4] * a[3] * a[13] +
              a[12] * a[1] * a[7] - a[12] * a[3] * a[5];
    inv[14] = -a[0] * a[5] * a[14] + a[0] * a[6] * a[13] + a[4] * a[1] * a[14] - a[4] * a[2] * a[13] -
              a[12] * a[1] * a[6] + a[12] * a[2] * a[5];
    inv[3] = -a[1] * a[6] * a[11] + a[1] * a[7] * a[10] + a[5] * a[2] * a[11] - a[5] * a[3] * a[10] -
             a[9] * a[2] * a[7] + a[9] * a[3] * a[6];
    inv[7] = a[0] * a[6] * a[11] - a[0] * a[7] * a[10] - a[4] * a[2] * a[11] + a[4] * a[3] * a[10] +
             a[8] * a[2] * a[7] - a[8] * a[3] * a[6];
    inv[11] = -a[0] * a[5] * a[11] + a[0] * a[7] * a[9] + a[4] * a[1] * a[11] - a[4] * a[3] * a[9] -
              a[8] * a[1] * a[7] + a[8] * a[3] * a[5];
    inv[15] = a[0] * a[5] * a[10] - a[0] * a[6] * a[9] - a[4] * a[1] * a[10] + a[4] * a[2] * a[9] +
              a[8] * a[1] * a[6] - a[8] * a[2] * a[5];
    const double det = a[0] * inv[0] + a[1] * inv[4] + a[2] * inv[8] + a[3] * inv[12];
    if (!(std::fabs(det) > 1e-30) || !std::isfinite(det)) return false;
    for (int i = 0; i < 16; ++i) out[i] = inv[i] / det;
    return true;
}

bool world_box(const double l2w[16], const BVHEntry& e, float4& lo, float4& hi) {
    const float c[2][3] = {{e.boundingCornerA.x, e.boundingCornerA.y, e.boundingCornerA.z},
                           {e.boundingCornerB.x, e.boundingCornerB.y, e.boundingCornerB.z}};
    double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
    for (int k = 0; k < 8; ++k) {
        const double p[3] = {c[k & 1][0], c[(k >> 1) & 1][1], c[(k >> 2) & 1][2]};
        for (int r = 0; r < 3; ++r) {  // column-major: M(r,col) = l2w[col*4 + r]
            const double w = l2w[r] * p[0] + l2w[4 + r] * p[1] + l2w[8 + r] * p[2] + l2w[12 + r];
            if (!std::isfinite(w)) return false;
            mn[r] = std::min(mn[r], w);
            mx[r] = std::max(mx[r], w);
        }
    }
    double size = 0.0, mag = 0.0;
    for (int r = 0; r < 3; ++r) {
        size = std::max(size, mx[r] - mn[r]);
        mag = std::max({mag, std::fabs(mn[r]), std::fabs(mx[r])});
    }
    const double pad = 1e-3 * size + 1e-4 * mag + 1e-5;
    lo = make_float4(float(mn[0] - pad), float(mn[1] - pad), float(mn[2] - pad), 0.0f);
    hi = make_float4(float(mx[0] + pad), float(mx[1] + pad), float(mx[2] + pad), 0.0f);
    return true;
}

bool mesh_cull_boxes(const hg_mat4& w2l, const BVHEntry& A, const BVHEntry& B, HgDevMesh& dm) {
    double a[16], l2w[16];
    for (int i = 0; i < 16; ++i) a[i] = w2l.m[i];
    if (!invert4(a, l2w)) return false;
    return world_box(l2w, A, dm.cull_a_lo, dm.cull_a_hi) && world_box(l2w, B, dm.cull_b_lo, dm.cull_b_hi);
}

// A mesh record's exact-cull boxes (its root's two children in world space) and cullable flag, from its matrix; all
// zero when not cullable, so a partial re-upload leaves no field of the previous matrix behind
void set_cull_boxes(const HalogenMeshData& m, const BVHEntry* blas, HgDevMesh& dm) {
    dm.cullable = 0;
    dm.cull_a_lo = dm.cull_a_hi = dm.cull_b_lo = dm.cull_b_hi = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const uint32_t off = m.accelerationBufferOffset;
    if (blas[off].triangleCount != 0) return;
    const BVHEntry& A = blas[off + blas[off].indexA];
    const BVHEntry& B = blas[off + blas[off].indexA + 1];
    if (mesh_cull_boxes(m.worldToLocal, A, B, dm)) dm.cullable = 1;
    else dm.cull_a_lo = dm.cull_a_hi = dm.cull_b_lo = dm.cull_b_hi = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

// The child-pair record layout (hg_device.h node_pair): q0 = (A.lo, refA), q1 = (A.hi, refB), q2 = (B.lo, -), q3 = (B.hi, -)
void put_pair(float4* r, const BVHEntry& A, const BVHEntry& B, uint32_t ra, uint32_t rb) {
    r[0] = f4(A.boundingCornerA.x, A.boundingCornerA.y, A.boundingCornerA.z, bits(ra));
    r[1] = f4(A.boundingCornerB.x, A.boundingCornerB.y, A.boundingCornerB.z, bits(rb));
    r[2] = f4(B.boundingCornerA.x, B.boundingCornerA.y, B.boundingCornerA.z, 0.0f);
    r[3] = f4(B.boundingCornerB.x, B.boundingCornerB.y, B.boundingCornerB.z, 0.0f);
}

// fn(begin, end) over [0, n) in contiguous chunks on the persistent host pool (hg_host_pool.h), at most `max_threads`
// chunks of at least `grain` items
template <class F>
void parallel_for(size_t n, size_t grain, int max_threads, F fn) {
    HgHostPool& pool = HgHostPool::get();
    const size_t t = std::max<size_t>(1, std::min<size_t>({size_t(max_threads), size_t(pool.threads()),
                                                           (n + grain - 1) / std::max<size_t>(grain, 1)}));
    if (t <= 1) {
        fn(size_t(0), n);
        return;
    }
    const size_t chunk = (n + t - 1) / t;
    pool.run(t, [&](size_t k) {
        const size_t b = std::min(n, k * chunk), e = std::min(n, b + chunk);
        if (b < e) fn(b, e);
    });
}

// Byte equality of two buffers, compared in parallel chunks (the scene's triangle array is 63 MB at C3)
bool same_bytes(const void* a, const void* b, size_t n) {
    if (n == 0) return true;
    std::atomic<bool> diff{false};
    parallel_for(n, size_t(4) << 20, kHostThreads, [&](size_t lo, size_t hi) {
        constexpr size_t step = size_t(1) << 20;
        for (size_t i = lo; i < hi && !diff.load(std::memory_order_relaxed); i += step)
            if (std::memcmp(static_cast<const char*>(a) + i, static_cast<const char*>(b) + i, std::min(step, hi - i)))
                diff.store(true, std::memory_order_relaxed);
    });
    return !diff.load();
}

void copy_bytes(std::vector<uint8_t>& dst, const void* src, size_t n) {
    dst.resize(n);
    if (n == 0) return;
    parallel_for(n, size_t(4) << 20, kHostThreads, [&](size_t lo, size_t hi) {
        std::memcpy(dst.data() + lo, static_cast<const char*>(src) + lo, hi - lo);
    });
}

int drain_events(hg_ctx* c) {
    if (c->pending.empty() && c->pending_trace.empty()) return HG_OK;
    HG_HIP(c, hipStreamSynchronize(c->stream));
    for (auto& pr : c->pending) {
        float ms = 0.0f;
        HG_HIP(c, hipEventElapsedTime(&ms, pr.first, pr.second));
        c->counters.kernel_ms += double(ms);
        c->free_events.push_back(pr);
    }
    // the launches' intervals relative to the first one pushed (which need not be the first to start: offsets can be
    // negative; the trace streams' events share the device clock); the batch ends at a synchronisation, so batches do
    // not overlap one another
    std::vector<std::pair<double, double>> iv;
    iv.reserve(c->pending_trace.size());
    for (auto& pr : c->pending_trace) {
        float ms = 0.0f, a = 0.0f;
        HG_HIP(c, hipEventElapsedTime(&ms, pr.first, pr.second));
        HG_HIP(c, hipEventElapsedTime(&a, c->pending_trace.front().first, pr.first));
        iv.emplace_back(double(a), double(a) + double(ms));
        c->counters.trace_ms += double(ms);
        c->counters.trace_launches++;
    }
    const double covered = hg_interval_union(std::move(iv));
    c->counters.trace_busy_ms += covered;
    for (auto& pr : c->pending_trace) c->free_events.push_back(pr);
    c->pending.clear();
    c->pending_trace.clear();
    return HG_OK;
}

int event_pair(hg_ctx* c, std::pair<hipEvent_t, hipEvent_t>& ev) {
    if (!c->free_events.empty()) {
        ev = c->free_events.back();
        c->free_events.pop_back();
        return HG_OK;
    }
    HG_HIP(c, hipEventCreate(&ev.first));
    HG_HIP(c, hipEventCreate(&ev.second));
    return HG_OK;
}

int ensure(hg_ctx* c, DevBuf& b, size_t bytes) {
    bytes = std::max<size_t>(bytes, 16);
    if (b.bytes >= bytes) return HG_OK;
    release(b);
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) return fail(c, HG_E_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    b.bytes = bytes;
    return HG_OK;
}

// The same in uncached device memory (MTYPE UC: no L2 holds its lines, so writes from one XCD are seen by loads from
// any other without cache maintenance): the render server's colour ring and frame counts, written by persistent
// waves and read by the gate and blend kernels while those waves still run
int ensure_uncached(hg_ctx* c, DevBuf& b, size_t bytes) {
    bytes = std::max<size_t>(bytes, 16);
    if (b.bytes >= bytes) return HG_OK;
    release(b);
    hipError_t e = hipExtMallocWithFlags(&b.p, bytes, hipDeviceMallocUncached);
    if (e != hipSuccess)
        return fail(c, HG_E_NOMEM, "hipExtMallocWithFlags(%zu, uncached) failed: %s", bytes, hipGetErrorString(e));
    b.bytes = bytes;
    return HG_OK;
}

double host_seconds() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---- the render server (hg_ctx::Server; device side hg_mega.hip kServer) ------------------------------------------
// The server closes itself after HG_OPT_SERVER_IDLE_US with nothing posted (the close handshake, hg_mega.hip sv_close:
// no host clock is involved in whether a post is taken).  A frame's gate gives up after 30 s, or at once when every
// wave of the server has left with the frame's count short: the frame is lost (reported, the accumulator invalid).
constexpr uint64_t kGateTimeoutTicks = 30ull * 100000000ull;  // 100-MHz s_memrealtime
// HG_OPT_SERVER_GATE_US, else HALOGEN_SERVER_GATE_TIMEOUT_MS (diagnostics: a shorter bound turns a stuck frame into an
// error fast), else 30 s
uint64_t gate_timeout_ticks(const hg_ctx* c) {
    if (c->sv.gate_us >= 0) return uint64_t(c->sv.gate_us) * 100ull;
    static const uint64_t t = [] {
        const char* e = std::getenv("HALOGEN_SERVER_GATE_TIMEOUT_MS");
        const long long ms = e ? std::atoll(e) : 0;
        return ms > 0 ? uint64_t(ms) * 100000ull : kGateTimeoutTicks;
    }();
    return t;
}

// HALOGEN_SERVER_TRACE=1: every server start, stop, post and refusal on stderr (diagnostics)
void sv_trace(const char* fmt, ...) {
    static const bool on = std::getenv("HALOGEN_SERVER_TRACE") != nullptr;
    if (!on) return;
    va_list ap;
    va_start(ap, fmt);
    std::fprintf(stderr, "[hg server %.6f] ", host_seconds());
    std::vfprintf(stderr, fmt, ap);
    std::fputc('\n', stderr);
    va_end(ap);
}

// A lost server frame, as its gate reported it in the host's lost-frame word (HG_SV_LOST | the accumulator epoch of the
// frame): the accumulator is invalid if the frame belongs to the current accumulation (a clear, a checkpoint load or a
// reallocation since has discarded it otherwise)
void server_note_lost(hg_ctx* c) {
    if (!c->sv.host) return;
    const unsigned long long w = __atomic_exchange_n(&c->sv.host[HG_SV_HOST_LOST], 0ull, __ATOMIC_SEQ_CST);
    if (!(w & HG_SV_LOST)) return;
    c->frames_lost++;
    sv_trace("a frame of accumulator epoch %u was lost (current epoch %u)", uint32_t(w), c->acc_epoch);
    if (uint32_t(w) == c->acc_epoch) c->acc_lost = true;
}
// The error of every entry point that renders into or reads the accumulator while it is invalid
int lost_check(hg_ctx* c) {
    server_note_lost(c);
    if (!c->acc_lost) return HG_OK;
    return fail(c, HG_E_FRAME_LOST, "a render server frame was lost (its gate gave up before the frame completed): the "
                                    "accumulation is invalid until hg_clear_accumulation or hg_set_accumulation");
}
// A new accumulation (clear, checkpoint load, reallocation), on the context stream after everything before it: lost
// frames before it no longer matter, and the blends after it run again
int reset_lost(hg_ctx* c) {
    server_note_lost(c);
    c->acc_epoch++;
    c->acc_lost = false;
    HG_HIP(c, hipMemsetAsync(c->lost.p, 0, sizeof(uint32_t), c->stream));
    return HG_OK;
}

// Stop the server: set the stop flag, the waves drain every frame posted and leave; wait (bounded) for the kernel.
int server_stop(hg_ctx* c) {
    hg_ctx::Server& S = c->sv;
    if (!S.running) return HG_OK;
    // the stop word carries the frames the host asked for: frames posted ahead of the calls (server_speculate) and not
    // yet claimed are abandoned (the waves' view drops to it, hg_mega.hip sv_view)
    __atomic_store_n(&S.host[HG_SV_HOST_POST], static_cast<unsigned long long>(S.committed) | HG_SV_STOP, __ATOMIC_SEQ_CST);
    const double t0 = host_seconds();
    sv_trace("stop: %u frames committed, %u posted", S.committed, S.posted);
    hipError_t q;
    while ((q = hipStreamQuery(S.stream)) == hipErrorNotReady) {
        if (host_seconds() - t0 > 60.0) {
            (void)hipGetLastError();
            return fail(c, HG_E_HIP, "render server did not stop within 60 s");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    (void)hipGetLastError();  // hipErrorNotReady is a status here
    S.running = false;
    sv_trace("stopped after %.3f ms (%s)", (host_seconds() - t0) * 1e3, hipGetErrorString(q));
#if HG_SV_DIAG_TIMES
    {  // (analysis builds) per frame: first claim and last count on the device clock (10 ns), host post time
        std::vector<unsigned long long> d(512);
        if (hipMemcpy(d.data(), static_cast<char*>(S.ctl.p) + HG_SV_DIAG_WORD * 4u, d.size() * 8u,
                      hipMemcpyDeviceToHost) == hipSuccess) {
            const unsigned long long t00 = ~d[0];
            for (uint32_t k = 0; k < std::min<uint32_t>(S.posted, 256u); ++k)
                sv_trace("frame %u: posted %+.3f ms (host), first claim %+.3f ms, last count %+.3f ms (device)", k,
                         (S.post_s[k] - S.post_s[0]) * 1e3, double(~d[2 * k] - t00) * 1e-5,
                         double(d[2 * k + 1] - t00) * 1e-5);
        }
    }
#endif
    if (q != hipSuccess) return fail(c, HG_E_HIP, "render server: %s", hipGetErrorString(q));
    return HG_OK;
}

// Wait for every stream of the context: the context stream and both trace streams (before device buffers that a
// trace in flight may read are changed or freed); the render server is stopped first
int quiesce(hg_ctx* c) {
    if (int rc = server_stop(c)) return rc;
    HG_HIP(c, hipStreamSynchronize(c->stream));
    if (c->rb_stream) HG_HIP(c, hipStreamSynchronize(c->rb_stream));
    for (hg_ctx::TraceLane& L : c->lanes)
        if (L.stream) HG_HIP(c, hipStreamSynchronize(L.stream));
    return HG_OK;
}

// Grow a trace stream's buffer; only when that buffer is not in use (quiesce first if it must move)
int ensure_quiet(hg_ctx* c, DevBuf& b, size_t bytes) {
    if (b.bytes >= std::max<size_t>(bytes, 16)) return HG_OK;
    if (int rc = quiesce(c)) return rc;
    return ensure(c, b, bytes);
}

int alloc_target(hg_ctx* c) {
    if (int rc = quiesce(c)) return rc;
    c->tiles_x = (c->W + HG_TILE - 1) / HG_TILE;
    c->tiles_y = (c->H + HG_TILE - 1) / HG_TILE;
    const int64_t total = int64_t(c->tiles_x) * c->tiles_y;
    c->n_local_tiles = total > c->rank ? int32_t((total - c->rank + c->n_ranks - 1) / c->n_ranks) : 0;
    for (hg_ctx::TraceLane& L : c->lanes) {
        L.tile_cost_valid = false;
        L.tile_order_valid = false;
        L.frames_since_order = 0;
    }
    c->sv.tile_cost_valid = false;  // (its buffer may be reallocated, or hold the old tiling's costs)
    if (int rc = reset_lost(c)) return rc;
    const size_t bytes = size_t(c->n_local_tiles) * 64 * sizeof(float4);
    c->rb_pending = 0;  // quiesced: begun readbacks are complete, and their images die with the old size or tiling
    c->rb_next = 0;
    release(c->acc);
    if (bytes) {
        hipError_t e = hipMalloc(&c->acc.p, bytes);
        if (e != hipSuccess) return fail(c, HG_E_NOMEM, "hipMalloc(accumulation %zu) failed", bytes);
        c->acc.bytes = bytes;
        HG_HIP(c, hipMemsetAsync(c->acc.p, 0, bytes, c->stream));
    }
    return HG_OK;
}


}  // namespace

extern "C" {

namespace {
// A trace stream (HG_LANE_STREAMS).  Plain streams share HIP's pool of GPU_MAX_HW_QUEUES (4) hardware queues with every
// other stream of the process; two trace streams on one queue serialise their launches.
hipError_t create_lane_stream(const hg_ctx* c, int lane, hipStream_t* s) {
    if (lane < HG_TRACE_LANES_BIG) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    std::vector<uint32_t> mask(size_t((c->n_cu + 31) / 32), 0u);
    for (int i = 0; i < c->n_cu; ++i) mask[size_t(i) / 32] |= 1u << (i % 32);
    // (CU-masked streams are blocking with respect to the legacy null stream, unlike the plain ones.)  Where the
    // runtime refuses CU masks, a plain stream: the same results, only the queue sharing above comes back.
    if (hipExtStreamCreateWithCUMask(s, uint32_t(mask.size()), mask.data()) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}
}  // namespace

int hg_abi_version(void) { return HG_ABI_VERSION; }

int hg_create(int device, hg_ctx** out) {
    if (!out) return HG_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return HG_E_HIP;
    if (device < 0 || device >= n) return HG_E_INVALID;
    hg_ctx* c = new hg_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->call_done[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->call_done[1], hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&c->counters_dev.p, 32 * sizeof(unsigned long long)) != hipSuccess) {
        delete c;
        return HG_E_HIP;
    }
    c->counters_dev.bytes = 32 * sizeof(unsigned long long);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        delete c;
        return HG_E_HIP;
    }
    c->n_cu = prop.multiProcessorCount;
    if (ensure_uncached(c, c->lost, 128) != HG_OK || hipMemset(c->lost.p, 0, 128) != hipSuccess ||
        hipMemset(c->counters_dev.p, 0, c->counters_dev.bytes) != hipSuccess) {
        hg_destroy(c);
        return HG_E_HIP;
    }
    for (int li = 0; li < HG_TRACE_LANES; ++li) {
        hg_ctx::TraceLane& L = c->lanes[li];
        if (create_lane_stream(c, li, &L.stream) != hipSuccess ||
            hipEventCreateWithFlags(&L.traced, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&L.blended, hipEventDisableTiming) != hipSuccess) {
            hg_destroy(c);
            return HG_E_HIP;
        }
    }
    *out = c;
    return HG_OK;
}

void hg_destroy(hg_ctx* c) {
    if (!c) return;
    c->pending_frames = 0;  // held frames are discarded: nothing can observe them after this call
    (void)hipSetDevice(c->device);
    (void)server_stop(c);
    sv_trace("destroy: server stopped");
    if (std::getenv("HALOGEN_SERVER_TRACE")) {
        unsigned long long w[4] = {};
        if (c->sv.ctl.p && hipMemcpyAsync(w, static_cast<char*>(c->sv.ctl.p) + HG_SV_EXIT_WORD * 4u, sizeof w,
                                          hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
            hipStreamSynchronize(c->stream) == hipSuccess)
            sv_trace("destroy: server waves out %llu of %llu", w[0] & 0xFFFFFFFFull, w[0] >> 32);
    }
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    sv_trace("destroy: context stream idle");
    for (hg_ctx::TraceLane& L : c->lanes)
        if (L.stream) (void)hipStreamSynchronize(L.stream);
    for (DevBuf* b : {&c->spheres, &c->meshes, &c->materials, &c->nodes, &c->leaves, &c->tris, &c->normals, &c->cube,
                      &c->acc, &c->counters_dev, &c->spill, &c->lost})
        release(*b);
    auto destroy_lanes = [c] {
        for (hg_ctx::TraceLane& L : c->lanes) {
            for (DevBuf* b : {&L.frame_color, &L.spill, &L.tile_cost, &L.tile_order, &L.order_scratch, &L.queue})
                release(*b);
            if (L.traced) (void)hipEventDestroy(L.traced);
            if (L.blended) (void)hipEventDestroy(L.blended);
            sv_trace("destroy: lane stream %p", static_cast<void*>(L.stream));
            if (L.stream) (void)hipStreamDestroy(L.stream);
        }
        sv_trace("destroy: trace streams destroyed");
    };
    // (analysis builds, HG_DIAG_TEARDOWN: HALOGEN_DIAG_TEARDOWN=server_first[,bufs_last][,host_last][,events_last]
    // destroys the server's stream before the trace streams, the order that hung in round 5, and defers the named
    // server resources past every stream destroy: tools/gpu_teardown.sh)
    bool server_first = false, bufs_last = false, host_last = false, events_last = false;
#if HG_DIAG_TEARDOWN
    if (const char* td = std::getenv("HALOGEN_DIAG_TEARDOWN")) {
        server_first = std::strstr(td, "server_first") != nullptr;
        bufs_last = std::strstr(td, "bufs_last") != nullptr;
        host_last = std::strstr(td, "host_last") != nullptr;
        events_last = std::strstr(td, "events_last") != nullptr;
    }
#endif
    hg_ctx::Server& S = c->sv;
    auto server_bufs = [&S] {
        for (DevBuf* b : {&S.ctl, &S.done, &S.ring, &S.spill, &S.tile_cost, &S.tile_order, &S.order_scratch}) release(*b);
        sv_trace("destroy: server buffers freed");
    };
    auto server_events = [&S] {
        for (hipEvent_t& e : S.blended)
            if (e) (void)hipEventDestroy(e);
        if (S.exited) (void)hipEventDestroy(S.exited);
        sv_trace("destroy: server events destroyed");
    };
    auto server_host = [&S] {
        if (S.host) (void)hipHostFree(S.host);
        sv_trace("destroy: server host word freed");
    };
    auto destroy_server = [&] {
        if (S.stream) (void)hipStreamSynchronize(S.stream);
        sv_trace("destroy: server stream idle");
        if (!bufs_last) server_bufs();
        if (!events_last) server_events();
        if (!host_last) server_host();
        if (S.stream) (void)hipStreamDestroy(S.stream);
        sv_trace("destroy: server stream destroyed");
    };
    // The server's stream after the trace streams: destroyed before them, the next hipStreamDestroy of a plain trace
    // stream hung in round 5 (DESIGN.md section 4.7 has what the analysis build found)
    if (server_first) destroy_server();
    destroy_lanes();
    if (!server_first) destroy_server();
    if (bufs_last) server_bufs();
    if (events_last) server_events();
    if (host_last) server_host();
    if (c->rb_stream) (void)hipStreamSynchronize(c->rb_stream);
    release(c->image);
    for (int k = 0; k < HG_READBACK_MAX; ++k) {
        release(c->rb_image[k]);
        if (c->rb_untiled[k]) (void)hipEventDestroy(c->rb_untiled[k]);
        if (c->image_host[k]) (void)hipHostFree(c->image_host[k]);
        if (c->image_copied[k]) (void)hipEventDestroy(c->image_copied[k]);
    }
    if (c->rb_stream) (void)hipStreamDestroy(c->rb_stream);
    for (auto& pr : c->pending_trace) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (auto& pr : c->pending) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (auto& pr : c->free_events) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (hipEvent_t e : c->call_done)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    sv_trace("destroy: done");
    delete c;
}

const char* hg_last_error(const hg_ctx* c) { return c ? c->err.c_str() : "null context"; }

int hg_upload_scene(hg_ctx* c, const HalogenSphere* spheres, int32_t n_spheres, const HalogenMeshData* meshes,
                    int32_t n_meshes, const PackedHalogenMaterial* materials, int32_t n_materials,
                    const HalogenTriangle* tris, int32_t n_tris, const BVHEntry* blas, int32_t n_nodes) {
    return hg_upload_scene_gen(c, 0, spheres, n_spheres, meshes, n_meshes, materials, n_materials, tris, n_tris, blas,
                               n_nodes);
}

int hg_upload_scene_gen(hg_ctx* c, uint64_t geometry_generation, const HalogenSphere* spheres, int32_t n_spheres,
                        const HalogenMeshData* meshes, int32_t n_meshes, const PackedHalogenMaterial* materials,
                        int32_t n_materials, const HalogenTriangle* tris, int32_t n_tris, const BVHEntry* blas,
                        int32_t n_nodes) {
    if (!c) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (n_spheres < 0 || n_meshes < 0 || n_materials < 0 || n_tris < 0 || n_nodes < 0)
        return fail(c, HG_E_INVALID, "negative count");
    if ((n_spheres && !spheres) || (n_meshes && !meshes) || (n_materials && !materials) || (n_tris && !tris) ||
        (n_nodes && !blas))
        return fail(c, HG_E_INVALID, "null array with non-zero count");
    // the traversal addresses nodes / triangles with 32-bit byte offsets (hg_device.h ld_off)
    if (n_nodes >= (1 << 26) || n_tris >= (1 << 28))
        return fail(c, HG_E_UNSUPPORTED, "scene too large: %d BLAS entries (max 2^26-1), %d triangles (max 2^28-1)",
                    n_nodes, n_tris);
    if (n_materials > 255)
        return fail(c, HG_E_UNSUPPORTED, "at most 255 materials (medium stack packs material indices in bytes)");
    // An upload of exactly the arrays already on the device changes nothing: the reference re-uploads every buffer
    // on each camera move (ClearAccumulation sets ObjectBuffersDirty, RP:262-268, 296-299), and the drop-in keeps that
    // call pattern.  Compared byte for byte against the retained host copies of the last upload (in parallel; ~3 ms
    // for C3's 80 MB), it skips the validation, the repack, the copies, the quiesce and the cost-order reset.
    const void* src[5] = {spheres, meshes, materials, tris, blas};
    const size_t bytes_in[5] = {size_t(n_spheres) * sizeof(HalogenSphere), size_t(n_meshes) * sizeof(HalogenMeshData),
                                size_t(n_materials) * sizeof(PackedHalogenMaterial),
                                size_t(n_tris) * sizeof(HalogenTriangle), size_t(n_nodes) * sizeof(BVHEntry)};
    bool same[5] = {false, false, false, false, false};
    // A caller-kept geometry generation equal to the last upload's vouches for the triangles and BVH entries (the C# /
    // C++ / Python passes bump it when RayTracingManager's mesh registry changes): no compare of those 78 MB (C3).
    const bool vouched = c->has_scene && geometry_generation != 0 && geometry_generation == c->geometry_gen;
    if (c->has_scene) {
        for (int k = 0; k < 5; ++k) same[k] = c->scene_copy[k].size() == bytes_in[k];
        for (int k = 0; k < 3; ++k)
            same[k] = same[k] && (!bytes_in[k] || !std::memcmp(c->scene_copy[k].data(), src[k], bytes_in[k]));
        for (int k = 3; k < 5; ++k)
            same[k] = same[k] && (vouched || same_bytes(c->scene_copy[k].data(), src[k], bytes_in[k]));
        if (same[0] && same[1] && same[2] && same[3] && same[4]) {
            c->scene_uploads_skipped++;
            c->scene_uploads_vouched += vouched ? 1u : 0u;
            // (compared equal: the caller's generation now names the device's geometry, so the next upload under it is
            // vouched for; without this, a first tagged upload of an untagged scene never let the next ones skip the
            // compare)
            c->geometry_gen = geometry_generation;
            return HG_OK;
        }
    }
    // ---- spheres
    std::vector<float4> sph(size_t(n_spheres) * 3);
    for (int i = 0; i < n_spheres; ++i) {
        const HalogenSphere& s = spheres[i];
        if (s.materialIndex >= uint32_t(n_materials))
            return fail(c, HG_E_INVALID, "sphere %d: materialIndex %u out of range", i, s.materialIndex);
        sph[3 * i] = f4(s.center.x, s.center.y, s.center.z, s.radius);
        sph[3 * i + 1] = f4(s.boundingCornerA.x, s.boundingCornerA.y, s.boundingCornerA.z, bits(s.materialIndex));
        sph[3 * i + 2] = f4(s.boundingCornerB.x, s.boundingCornerB.y, s.boundingCornerB.z, 0.0f);
    }
    // ---- materials
    std::vector<float4> mat(size_t(n_materials) * 5);
    for (int i = 0; i < n_materials; ++i) {
        const PackedHalogenMaterial& m = materials[i];
        mat[5 * i] = f4(m.albedo.x, m.albedo.y, m.albedo.z, m.albedo.w);
        mat[5 * i + 1] = f4(m.specularAlbedo.x, m.specularAlbedo.y, m.specularAlbedo.z, m.metallic);
        // emissive.rgb * emissive.a (:901) and roughness^2 (:699) are the kernel's own operations done once here
        mat[5 * i + 2] = f4(m.emissive.x * m.emissive.w, m.emissive.y * m.emissive.w, m.emissive.z * m.emissive.w,
                            m.roughness);
        mat[5 * i + 3] = f4(m.rayMedium.absorption.x, m.rayMedium.absorption.y, m.rayMedium.absorption.z,
                            m.rayMedium.indexOfRefraction);
        mat[5 * i + 4] = f4(bits(m.rayMedium.priority), bits(m.rayMedium.materialID), m.roughness * m.roughness, 0.0f);
    }
    // Partial re-upload: the triangles and the BVH entries are the last upload's and every mesh keeps its buffer
    // offsets (objects moved, or materials / spheres changed): the node records, leaves, triangles and normals on the
    // device stay; only the mesh table (world->local matrices, materials, exact-cull boxes), spheres and materials are
    // rebuilt and copied.  Same device contents as a full upload of these arrays.
    bool partial = c->has_scene && same[3] && same[4] && size_t(n_meshes) == c->dev_meshes.size() &&
                   c->scene_copy[1].size() == bytes_in[1];
    for (int mi = 0; partial && mi < n_meshes; ++mi) {
        const HalogenMeshData& o = reinterpret_cast<const HalogenMeshData*>(c->scene_copy[1].data())[mi];
        partial = o.triangleBufferOffset == meshes[mi].triangleBufferOffset &&
                  o.accelerationBufferOffset == meshes[mi].accelerationBufferOffset;
    }
    if (partial) {
        std::vector<HgDevMesh> dm = c->dev_meshes;
        for (int mi = 0; mi < n_meshes; ++mi) {
            const HalogenMeshData& m = meshes[mi];
            if (m.materialIndex >= uint32_t(n_materials))
                return fail(c, HG_E_INVALID, "mesh %d: materialIndex %u out of range", mi, m.materialIndex);
            std::memcpy(dm[mi].w2l, m.worldToLocal.m, sizeof dm[mi].w2l);
            dm[mi].material = m.materialIndex;
            set_cull_boxes(m, blas, dm[mi]);
        }
        if (int rc = set_device(c)) return rc;
        if (int rc = quiesce(c)) return rc;  // no trace in flight reads the buffers replaced below
        c->has_scene = false;
        int rc;
        if ((rc = upload(c, c->spheres, sph.data(), sph.size() * sizeof(float4)))) return rc;
        if ((rc = upload(c, c->materials, mat.data(), mat.size() * sizeof(float4)))) return rc;
        if ((rc = upload(c, c->meshes, dm.data(), dm.size() * sizeof(HgDevMesh)))) return rc;
        for (int k = 0; k < 3; ++k) copy_bytes(c->scene_copy[k], src[k], bytes_in[k]);
        HG_HIP(c, hipStreamSynchronize(c->stream));
        c->dev_meshes.swap(dm);
        c->scene_uploads++;
        c->scene_uploads_partial++;
        c->scene_uploads_vouched += vouched ? 1u : 0u;
        c->geometry_gen = geometry_generation;
        c->n_spheres = n_spheres;
        c->n_meshes = n_meshes;
        c->n_materials = n_materials;
        c->has_scene = true;
        return HG_OK;
    }
    if (int rc = set_device(c)) return rc;
    if (int rc = quiesce(c)) return rc;  // no trace in flight reads the buffers replaced below
    c->has_scene = false;
    for (auto& v : c->scene_copy) v.clear();

    // ---- triangles (independent per triangle: parallel)
    const size_t nt = size_t(n_tris);
    std::vector<float> t9(nt * 9);  // (v0, e1, e2) of tri_load, packed per triangle
    std::vector<float4> nrm(nt * 3);
    parallel_for(nt, 32768, kHostThreads, [&](size_t lo, size_t hi) {
        for (size_t t = lo; t < hi; ++t) {
            const HalogenTriangle& h = tris[t];
            const float e1x = h.pointB.x - h.pointA.x, e1y = h.pointB.y - h.pointA.y, e1z = h.pointB.z - h.pointA.z;
            const float e2x = h.pointC.x - h.pointA.x, e2y = h.pointC.y - h.pointA.y, e2z = h.pointC.z - h.pointA.z;
            const float v[9] = {h.pointA.x, h.pointA.y, h.pointA.z, e1x, e1y, e1z, e2x, e2y, e2z};
            std::memcpy(&t9[9 * t], v, sizeof v);
            nrm[3 * t] = f4(h.normalA.x, h.normalA.y, h.normalA.z, 0.0f);
            nrm[3 * t + 1] = f4(h.normalB.x - h.normalA.x, h.normalB.y - h.normalA.y, h.normalB.z - h.normalA.z, 0.0f);
            nrm[3 * t + 2] = f4(h.normalC.x - h.normalA.x, h.normalC.y - h.normalA.y, h.normalC.z - h.normalA.z, 0.0f);
        }
    });
    // ---- BLAS, pass 1: validate every mesh's tree by DFS (ranges, depth, sharing between meshes)
    std::vector<int64_t> owner(size_t(n_nodes), -1);  // (accOffset << 32 | triOffset) that produced the entry
    std::vector<HgDevMesh> dm(static_cast<size_t>(n_meshes));
    uint32_t max_depth = 0;
    std::vector<std::pair<uint32_t, uint32_t>> dfs;
    for (int mi = 0; mi < n_meshes; ++mi) {
        const HalogenMeshData& m = meshes[mi];
        if (m.materialIndex >= uint32_t(n_materials))
            return fail(c, HG_E_INVALID, "mesh %d: materialIndex %u out of range", mi, m.materialIndex);
        const uint32_t off = m.accelerationBufferOffset, toff = m.triangleBufferOffset;
        if (off >= uint32_t(n_nodes)) return fail(c, HG_E_INVALID, "mesh %d: accelerationBufferOffset out of range", mi);
        const int64_t key = (int64_t(off) << 32) | int64_t(toff);
        dfs.assign(1, {off, 0u});
        while (!dfs.empty()) {
            auto [g, depth] = dfs.back();
            dfs.pop_back();
            if (depth + 2 > kMaxStack)
                return fail(c, HG_E_UNSUPPORTED, "mesh %d: BLAS deeper than %u levels (or cyclic)", mi, kMaxStack - 2);
            max_depth = std::max(max_depth, depth);
            if (owner[g] != -1 && owner[g] != key)
                return fail(c, HG_E_UNSUPPORTED, "BLAS entry %u shared by meshes with different offsets", g);
            owner[g] = key;
            const BVHEntry& e = blas[g];
            if (e.triangleCount > 0) {
                if (uint64_t(toff) + e.indexA + e.triangleCount > uint64_t(n_tris))
                    return fail(c, HG_E_INVALID, "mesh %d: leaf %u references triangles out of range", mi, g);
            } else {
                const uint64_t a = uint64_t(off) + e.indexA;
                if (a + 1 >= uint64_t(n_nodes))
                    return fail(c, HG_E_INVALID, "mesh %d: node %u has children out of range", mi, g);
                dfs.push_back({uint32_t(a + 1), depth + 1});
                dfs.push_back({uint32_t(a), depth + 1});
            }
        }
    }
    // ---- BLAS, pass 2: device layout.  Inner nodes get a child-pair record (both children's boxes + refs, 64 B),
    // leaves an entry of the leaf table.  Records are numbered in depth-first pre-order of sibling pairs: the two
    // children of a node sit in one 128-B line (the far sibling, popped later, is usually still cached) and a
    // subtree's records are contiguous.  Traversal follows refs only, so visit order and results are unchanged.
    std::vector<uint32_t> dref(size_t(n_nodes), HG_NONE);  // device ref of each reference BVH entry
    std::vector<float4> rec;
    std::vector<uint2> leaf;
    rec.reserve(size_t(n_nodes) * 4 + 8);
    auto new_record = [&]() {
        rec.resize(rec.size() + 4, f4(0, 0, 0, 0));
        return uint32_t(rec.size() / 4 - 1);
    };
    std::vector<uint32_t> expand;
    for (int mi = 0; mi < n_meshes; ++mi) {
        const HalogenMeshData& m = meshes[mi];
        const uint32_t off = m.accelerationBufferOffset, toff = m.triangleBufferOffset;
        auto ref_for = [&](uint32_t g, bool with_sibling_pad) -> uint32_t {  // assigns a device ref on first use
            if (dref[g] != HG_NONE) return dref[g];
            const BVHEntry& e = blas[g];
            if (e.triangleCount > 0) {
                const uint64_t first = uint64_t(toff) + e.indexA;
                if (e.triangleCount <= HG_LEAF_INLINE_MAX && first < HG_LEAF_PAYLOAD) {  // never encodes HG_NONE
                    dref[g] = HG_LEAF_BIT | (e.triangleCount << HG_LEAF_CNT_SHIFT) | uint32_t(first);
                } else {
                    if (leaf.size() > HG_LEAF_PAYLOAD) return HG_NONE;  // reported below
                    dref[g] = HG_LEAF_BIT | uint32_t(leaf.size());
                    leaf.push_back(make_uint2(uint32_t(first), e.triangleCount));
                }
            } else {
                if (with_sibling_pad && (rec.size() / 4) % 2 == 1) new_record();  // pair starts on an even record
                dref[g] = new_record();
                expand.push_back(g);
            }
            return dref[g];
        };
        const uint32_t root = ref_for(off, false);
        if (root == HG_NONE) return fail(c, HG_E_UNSUPPORTED, "too many large BLAS leaves");
        while (!expand.empty()) {
            const uint32_t g = expand.back();
            expand.pop_back();
            const uint32_t a = off + blas[g].indexA;
            const bool both_new = dref[a] == HG_NONE && dref[a + 1] == HG_NONE && blas[a].triangleCount == 0 &&
                                  blas[a + 1].triangleCount == 0;
            const size_t mark = expand.size();
            const uint32_t ra = ref_for(a, both_new);
            const uint32_t rb = ref_for(a + 1, false);
            if (ra == HG_NONE || rb == HG_NONE) return fail(c, HG_E_UNSUPPORTED, "too many large BLAS leaves");
            if (expand.size() == mark + 2) std::swap(expand[mark], expand[mark + 1]);  // expand child A first
            const BVHEntry& A = blas[a];
            const BVHEntry& B = blas[a + 1];
            put_pair(&rec[4 * size_t(dref[g])], A, B, ra, rb);
        }
        std::memcpy(dm[mi].w2l, m.worldToLocal.m, sizeof dm[mi].w2l);
        dm[mi].root_ref = root;
        dm[mi].tri_offset = toff;
        dm[mi].material = m.materialIndex;
        set_cull_boxes(m, blas, dm[mi]);
    }
    if (rec.size() / 4 >= (size_t(1) << 26))
        return fail(c, HG_E_UNSUPPORTED, "BLAS too large: %zu device node records", rec.size() / 4);
    if (rec.empty()) new_record();
    if (leaf.empty()) leaf.push_back(make_uint2(0, 0));
    c->stack_depth = std::max<uint32_t>(2u, (max_depth + 2 + 1) & ~1u);

    int rc;
    if ((rc = upload(c, c->spheres, sph.data(), sph.size() * sizeof(float4)))) return rc;
    if ((rc = upload(c, c->materials, mat.data(), mat.size() * sizeof(float4)))) return rc;
    if ((rc = upload(c, c->meshes, dm.data(), dm.size() * sizeof(HgDevMesh)))) return rc;
    if ((rc = upload(c, c->nodes, rec.data(), rec.size() * sizeof(float4)))) return rc;
    if ((rc = upload(c, c->leaves, leaf.data(), leaf.size() * sizeof(uint2)))) return rc;
    if ((rc = upload(c, c->tris, t9.data(), t9.size() * sizeof(float)))) return rc;
    if ((rc = upload(c, c->normals, nrm.data(), nrm.size() * sizeof(float4)))) return rc;
    // the retained copies the next upload compares against (while the device copies run)
    for (int k = 0; k < 5; ++k) copy_bytes(c->scene_copy[k], src[k], bytes_in[k]);
    c->dev_meshes = dm;
    HG_HIP(c, hipStreamSynchronize(c->stream));  // host staging vectors die at return
    c->geometry_gen = geometry_generation;
    c->scene_uploads++;
    c->n_spheres = n_spheres;
    c->n_meshes = n_meshes;
    c->n_materials = n_materials;
    c->n_tris = n_tris;
    c->n_nodes = n_nodes;
    c->has_scene = true;
    return HG_OK;
}

int hg_upload_cubemap(hg_ctx* c, int32_t face_size, int32_t n_mips, const float* texels, size_t n_floats) {
    if (!c) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (face_size <= 0 || n_mips <= 0 || n_mips > HG_MAX_CUBE_MIPS || !texels)
        return fail(c, HG_E_INVALID, "bad cubemap shape");
    uint64_t need = 0;
    for (int m = 0; m < n_mips; ++m) {
        c->cube_mip_offset[m] = uint32_t(need / 4);
        const uint64_t s = std::max(1, face_size >> m);
        need += 6ull * s * s * 4ull;
    }
    if (need != n_floats) return fail(c, HG_E_INVALID, "cubemap has %zu floats, expected %llu", n_floats,
                                      (unsigned long long)need);
    if (int rc = set_device(c)) return rc;
    if (int rc = quiesce(c)) return rc;
    if (int rc = upload(c, c->cube, texels, n_floats * sizeof(float))) return rc;
    HG_HIP(c, hipStreamSynchronize(c->stream));
    c->cube_size = face_size;
    c->cube_mips = n_mips;
    return HG_OK;
}

int hg_set_params(hg_ctx* c, const hg_params* p) {
    if (!c || !p) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (p->samplesPerPixel < 1) return fail(c, HG_E_INVALID, "samplesPerPixel must be >= 1");
    if (!(p->screenParameters.x >= 1.0f) || !(p->screenParameters.y >= 1.0f))
        return fail(c, HG_E_INVALID, "screenParameters must be >= 1");
    c->params = *p;
    c->has_params = true;
    return HG_OK;
}

int hg_resize(hg_ctx* c, int32_t width, int32_t height) {
    if (!c) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (width <= 0 || height <= 0 || int64_t(width) * height > (int64_t(1) << 31))
        return fail(c, HG_E_INVALID, "bad target size %dx%d", width, height);
    if (int rc = set_device(c)) return rc;
    c->W = width;
    c->H = height;
    return alloc_target(c);
}

int hg_set_tiling(hg_ctx* c, int32_t rank, int32_t n_ranks) {
    if (!c) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(c, HG_E_INVALID, "bad tiling %d/%d", rank, n_ranks);
    if (int rc = set_device(c)) return rc;
    c->rank = rank;
    c->n_ranks = n_ranks;
    return c->W > 0 ? alloc_target(c) : HG_OK;
}

int hg_clear_accumulation(hg_ctx* c) {
    if (!c) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (int rc = set_device(c)) return rc;
    if (c->acc.p) HG_HIP(c, hipMemsetAsync(c->acc.p, 0, c->acc.bytes, c->stream));
    return reset_lost(c);
}

}  // extern "C"

namespace {

// Validation of an hg_render call against the context's state (at the call, so that errors come from the call itself)
int render_check(hg_ctx* c, int32_t n_frames) {
    if (!c->has_scene) return fail(c, HG_E_NOSCENE, "hg_upload_scene not called");
    if (!c->has_params) return fail(c, HG_E_INVALID, "hg_set_params not called");
    if (c->W <= 0) return fail(c, HG_E_NOTARGET, "hg_resize not called");
    if (n_frames < 0) return fail(c, HG_E_INVALID, "n_frames < 0");
    const hg_params& p = c->params;
    if (int32_t(p.screenParameters.x) != c->W || int32_t(p.screenParameters.y) != c->H)
        return fail(c, HG_E_INVALID, "screenParameters (%g,%g) != target %dx%d", p.screenParameters.x,
                    p.screenParameters.y, c->W, c->H);
    const int32_t ns = int32_t(p.bufferCounts.x), nm = int32_t(p.bufferCounts.y);
    if (ns < 0 || ns > c->n_spheres || nm < 0 || nm > c->n_meshes)
        return fail(c, HG_E_INVALID, "bufferCounts (%d,%d) exceed uploaded (%d,%d)", ns, nm, c->n_spheres, c->n_meshes);
    return HG_OK;
}

// The server can take the frame of FrameCount `fc` next: running, started with these parameters and options, `fc`
// continuing its chain, room left in its lifetime's unit numbering, not closing (sv_close) and its kernel still resident
bool server_continues(hg_ctx* c, int32_t fc) {
    const hg_ctx::Server& S = c->sv;
    if (!S.running) return false;
    hg_params p = c->params;
    p.frameCount = S.params.frameCount;
    if (std::memcmp(&p, &S.params, sizeof p) != 0 || int64_t(fc) != int64_t(S.params.frameCount) + int64_t(S.committed) ||
        S.kernel_variant != c->kernel || S.descent_t != c->descent_t || S.posted >= S.cap ||
        __atomic_load_n(&S.host[HG_SV_HOST_CLOSING], __ATOMIC_SEQ_CST) != 0ull)
        return false;
    const hipError_t q = hipStreamQuery(S.stream);
    (void)hipGetLastError();
    return q == hipErrorNotReady;
}

// Launch the server for the frames from FrameCount `fc`: kp is the launch's parameter block as render_now built it.  HG_E_UNSUPPORTED when the device gives no stream with a hardware queue of its own (the server's
// gates on the context stream must never queue behind it): the caller launches per call instead.
// HALOGEN_SERVER_SERIAL=1: every gate waits for its server lifetime's end (a profiling aid for profilers that run one
// kernel at a time; the frames are then blended only after the lifetime closes, on idle or at a stop)
bool server_serial() {
    static const bool on = [] {
        const char* e = std::getenv("HALOGEN_SERVER_SERIAL");
        return e && std::atoi(e) == 1;
    }();
    return on;
}

int server_start(hg_ctx* c, const HgKernelParams& kp_in, int32_t fc) {
    hg_ctx::Server& S = c->sv;
    if (!S.stream) {
        std::vector<uint32_t> mask(size_t((c->n_cu + 31) / 32), 0u);
        for (int i = 0; i < c->n_cu; ++i) mask[size_t(i) / 32] |= 1u << (i % 32);
        if (hipExtStreamCreateWithCUMask(&S.stream, uint32_t(mask.size()), mask.data()) != hipSuccess) {
            (void)hipGetLastError();
            S.stream = nullptr;
            c->server_on = 0;
            return HG_E_UNSUPPORTED;
        }
        for (hipEvent_t& e : S.blended) HG_HIP(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HG_HIP(c, hipEventCreateWithFlags(&S.exited, hipEventDisableTiming));
        // coherent (fine-grained) pinned memory: the pollers' system-scope loads of the post word read host memory
        // itself (measured the same as the default pinned memory, tools/sweeps/sweep_r05_server.txt; this is the
        // memory type whose coherence the loads rely on)
        HG_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&S.host), 256, hipHostMallocMapped | hipHostMallocCoherent));
        for (int k = 0; k < 4; ++k) S.host[k] = 0ull;
    }
    const uint32_t tiles = uint32_t(c->n_local_tiles);
    const size_t per_frame = size_t(tiles) * 64u * sizeof(float4);
    uint32_t ring = HG_SV_RING;
    while (ring > 2u && size_t(ring) * per_frame > (size_t(2) << 30)) ring >>= 1;
    // waves per SIMD: HG_SV_WAVES, the kernel's occupancy (HALOGEN_SERVER_WAVES overrides, 1..HG_STREAM_WAVES, for A/B)
    static const uint32_t sv_waves = [] {
        const char* e = std::getenv("HALOGEN_SERVER_WAVES");
        const int v = e ? std::atoi(e) : 0;
        return uint32_t(v >= 1 && v <= HG_STREAM_WAVES ? v : HG_SV_WAVES);
    }();
    const uint32_t slots = uint32_t(c->n_cu) * 4u * sv_waves;
    const uint32_t grid = std::min(tiles, slots);
    const uint32_t lds_part = HG_STREAM_LDS_STACK;
    const size_t spill_bytes = kp_in.stack_depth > lds_part ? size_t(grid) * 64u * (kp_in.stack_depth - lds_part) * 4u : 0;
    const size_t tb = size_t(tiles) * sizeof(uint32_t);
    // the last lifetime's gates and blends on the context stream read its ring and counts: everything below runs after
    // them (an event, no host wait) unless a buffer must move (then the context stream is drained first)
    if (S.ring.bytes < size_t(ring) * per_frame || S.done.bytes < size_t(ring) * 128u)
        HG_HIP(c, hipStreamSynchronize(c->stream));
    int rc = ensure_uncached(c, S.ring, size_t(ring) * per_frame);
    if (!rc) rc = ensure_uncached(c, S.done, size_t(ring) * 128u);
    if (!rc) rc = ensure_uncached(c, S.ctl, HG_SV_CTL_BYTES);  // (polled by scalar loads: hg_mega.hip sv_sload)
    if (!rc && spill_bytes) rc = ensure(c, S.spill, spill_bytes);
    // the cost order only with HG_SV_COST_ORDER: the server's frames overlap, so no frame's end waits on its longest
    // tiles, and raster order keeps a claim's consecutive tiles together (HG_SV_COST_ORDER in hg_layout.h)
    const bool ordered = c->tile_order_on && HG_SV_COST_ORDER;
    if (!rc && ordered) rc = ensure(c, S.tile_cost, 2 * tb);
    if (!rc && ordered) rc = ensure(c, S.tile_order, tb);
    const size_t osb = hg_order_scratch_bytes(tiles);
    if (!rc && ordered && S.order_scratch.bytes < osb) {
        rc = ensure(c, S.order_scratch, osb);
        if (!rc && hipMemsetAsync(S.order_scratch.p, 0, S.order_scratch.bytes, S.stream) != hipSuccess)
            rc = fail(c, HG_E_HIP, "hipMemsetAsync(server order scratch) failed");
    }
    if (rc) return rc;
    // The counts and heads are zeroed on the context stream: after the last lifetime's gates and blends, and before
    // this lifetime's gates, which are queued there too (zeroed on the server's stream instead, a new gate could read
    // the last lifetime's count of its ring slot before the zeroing and pass at once)
    HG_HIP(c, hipMemsetAsync(S.ctl.p, 0, HG_SV_CTL_BYTES, c->stream));
    HG_HIP(c, hipMemsetAsync(S.done.p, 0, size_t(ring) * 128u, c->stream));
    std::pair<hipEvent_t, hipEvent_t> ev;
    if (int r = event_pair(c, ev)) return r;
    HG_HIP(c, hipEventRecord(ev.first, c->stream));
    HG_HIP(c, hipStreamWaitEvent(S.stream, ev.first, 0));
    c->free_events.push_back(ev);
    HgKernelParams kp = kp_in;
    kp.tile_order = nullptr;
    kp.tile_cost = nullptr;
    if (ordered) {
        kp.tile_cost = static_cast<unsigned long long*>(S.tile_cost.p);
        if (S.tile_cost_valid) {  // the cost order of the last lifetime's frames
            HG_HIP(c, hg_launch_order_tiles(kp.tile_cost, static_cast<uint32_t*>(S.tile_order.p), tiles, S.order_scratch.p,
                                            static_cast<unsigned long long*>(c->counters_dev.p) + 18, S.stream));
            kp.tile_order = static_cast<const uint32_t*>(S.tile_order.p);
        } else {
            HG_HIP(c, hipMemsetAsync(kp.tile_cost, 0, size_t(tiles) * sizeof(unsigned long long), S.stream));
            S.tile_cost_valid = true;
        }
    }
    kp.frame_color = static_cast<float4*>(S.ring.p);
    kp.frames_done = static_cast<uint32_t*>(S.done.p);
    kp.queue = static_cast<uint32_t*>(S.ctl.p);
    kp.resident_waves = slots;
    kp.wave_units = 1;
    kp.spill = spill_bytes ? static_cast<uint32_t*>(S.spill.p) : nullptr;
    kp.spill_stride = grid * 64u;
    kp.first_frame = fc;
    kp.n_frames = 1;
    kp.frame_split = 1;
    kp.accumulate = 1;
    void* post = nullptr;
    HG_HIP(c, hipHostGetDevicePointer(&post, S.host, 0));
    kp.sv_post = static_cast<const unsigned long long*>(post);
    kp.sv_ring = ring;
    kp.sv_frames_cap = std::min<uint32_t>(1u << 24, uint32_t((uint64_t(1) << 31) / std::max<uint32_t>(tiles, 1u)));
    kp.sv_idle_ticks = uint32_t(std::min<uint64_t>(uint64_t(S.idle_us) * 100ull, 0xFFFFFFFFull));
    if ((tiles & (tiles - 1u)) == 0u) {  // unit -> frame (hg_mega.hip sv_frame): a shift, or a multiply-high and a shift
        kp.sv_div_magic = 0u;
        kp.sv_div_shift = uint32_t(__builtin_ctz(tiles));
    } else {
        const uint32_t l = 31u - uint32_t(__builtin_clz(tiles));
        kp.sv_div_magic = uint32_t(((uint64_t(1) << (32 + l)) + tiles - 1u) / tiles);
        kp.sv_div_shift = l;
    }
    // (the lost-frame word is not reset: a gate of the last lifetime may still report into it)
    __atomic_store_n(&S.host[HG_SV_HOST_POST], 0ull, __ATOMIC_SEQ_CST);
    __atomic_store_n(&S.host[HG_SV_HOST_CLOSING], 0ull, __ATOMIC_SEQ_CST);
    __atomic_store_n(&S.host[HG_SV_HOST_CLOSED], 0ull, __ATOMIC_SEQ_CST);
    HG_HIP(c, hg_launch_mega_stream(kp, 64, c->counters_on != 0, S.stream, true));
    if (server_serial()) HG_HIP(c, hipEventRecord(S.exited, S.stream));
    S.running = true;
    S.ring_n = ring;
    S.posted = 0;
    S.committed = 0;
    S.cap = kp.sv_frames_cap;
    for (uint32_t k = 0; k < HG_SV_RING; ++k) {
        S.uses[k] = 0;
        S.blend_valid[k] = false;
    }
    S.params = c->params;
    S.params.frameCount = fc;
    S.kernel_variant = c->kernel;
    S.descent_t = c->descent_t;
    S.kp = kp;
    c->server_launches++;
    sv_trace("start: FrameCount %d, %u tiles, ring %u, grid %u", fc, tiles, ring, grid);
    return HG_OK;
}

// Post frame k = S.posted to the server: the host's half of the close handshake (hg_mega.hip sv_close).  Raise the post
// word, then read the closing word.  Not raised: the post is taken (a wave that closes later reads the post word after
// this store).  Raised: the post is taken only if the closing wave's read of the post word included it (the close
// word); else HG_E_UNSUPPORTED, nothing posted: the caller restarts the server and posts there.  The ring slot must be
// free (its frame ring_n back blended).
int server_post_frame(hg_ctx* c) {
    hg_ctx::Server& S = c->sv;
    const uint32_t k = S.posted, s = k & (S.ring_n - 1u);
    __atomic_store_n(&S.host[HG_SV_HOST_POST], static_cast<unsigned long long>(k + 1u), __ATOMIC_SEQ_CST);
    if (__atomic_load_n(&S.host[HG_SV_HOST_CLOSING], __ATOMIC_SEQ_CST) != 0ull) {
        // the closing wave publishes the post word it read right after reading it (bounded wait: a wave that raised
        // the closing word is running its next few instructions)
        unsigned long long fin;
        const double t0 = host_seconds();
        while (!((fin = __atomic_load_n(&S.host[HG_SV_HOST_CLOSED], __ATOMIC_SEQ_CST)) & HG_SV_CLOSED)) {
            if (host_seconds() - t0 > 10.0) return fail(c, HG_E_HIP, "render server: the closing wave never published");
            std::this_thread::yield();
        }
        if (uint32_t(fin) < k + 1u) {
            c->server_refused++;
            sv_trace("post %u: refused (the server closed at %u frames)", k, uint32_t(fin));
            return HG_E_UNSUPPORTED;
        }
        sv_trace("post %u: taken by a closing server", k);
    }
    S.uses[s]++;
    S.posted = k + 1u;
#if HG_SV_DIAG_TIMES
    if (k < 256u) S.post_s[k] = host_seconds();
#endif
    return HG_OK;
}

// The frame the host asks for next (FrameCount = first + committed): posted now, unless it was posted ahead
// (server_speculate), then its gate + blend on the context stream (in frame order, like every other blend).  Frames run
// at most ring_n ahead of their blends (the host waits for the blend of the frame ring_n back before reusing its ring
// slot).  HG_E_UNSUPPORTED: the post was refused (a closing server), nothing queued.
int server_commit(hg_ctx* c) {
    hg_ctx::Server& S = c->sv;
    const uint32_t k = S.committed, s = k & (S.ring_n - 1u);
    if (k == S.posted) {
        if (S.blend_valid[s]) {
            sv_trace("post %u: waiting for the blend of frame %u", k, k - S.ring_n);
            HG_HIP(c, hipEventSynchronize(S.blended[s]));
        }
        if (int rc = server_post_frame(c)) return rc;
    }
    const uint32_t tiles = uint32_t(c->n_local_tiles), n_slots = tiles * 64u;
    void* err = nullptr;
    HG_HIP(c, hipHostGetDevicePointer(&err, S.host + HG_SV_HOST_LOST, 0));
    if (server_serial()) HG_HIP(c, hipStreamWaitEvent(c->stream, S.exited, 0));
    HG_HIP(c, hg_launch_server_frame(static_cast<float4*>(c->acc.p),
                                     static_cast<const float4*>(S.ring.p) + size_t(s) * n_slots, n_slots,
                                     S.kp.first_frame + int32_t(k), static_cast<const uint32_t*>(S.done.p) + 32u * s,
                                     S.uses[s] * tiles, gate_timeout_ticks(c),
                                     reinterpret_cast<const unsigned long long*>(static_cast<const uint32_t*>(S.ctl.p) +
                                                                                 HG_SV_EXIT_WORD),
                                     static_cast<uint32_t*>(c->lost.p), static_cast<unsigned long long*>(err),
                                     c->acc_epoch, c->stream));
    HG_HIP(c, hipEventRecord(S.blended[s], c->stream));
    S.blend_valid[s] = true;
    S.committed = k + 1u;
    c->server_frames++;
    sv_trace("committed %u (slot %u, target %u)", k, s, S.uses[s] * tiles);
    return HG_OK;
}

// Frames traced ahead of the host's calls (HG_OPT_SERVER_AHEAD, with the counters off): the next frames of the same
// parameters and FrameCount chain are posted without a gate or blend, never waiting (a ring slot whose blend has not
// run stops it).  A call that continues the chain commits them (server_commit); anything else stops the server and
// abandons those not yet claimed.  The host's display of frame k then waits only for frame k's gate, blend and copy:
// frame k + 1 is already being traced.  Same images (a frame is blended only when the host asks for it).
void server_speculate(hg_ctx* c) {
    hg_ctx::Server& S = c->sv;
    if (c->sv_ahead <= 0 || c->counters_on) return;
    const uint32_t ahead = std::min<uint32_t>(uint32_t(c->sv_ahead), S.ring_n - 2u);
    while (S.posted < S.committed + ahead && S.posted < S.cap) {
        const uint32_t s = S.posted & (S.ring_n - 1u);
        if (S.blend_valid[s]) {
            const hipError_t q = hipEventQuery(S.blended[s]);
            (void)hipGetLastError();  // hipErrorNotReady is a status here
            if (q != hipSuccess) return;
        }
        if (server_post_frame(c) != HG_OK) return;  // (refused: the next call restarts the server)
        c->server_ahead_posts++;
    }
}

// n_frames frames from FrameCount = params.frameCount through the server (started or restarted as needed).  A first
// HG_E_UNSUPPORTED (no stream of its own) falls back to launches; nothing was posted then.  A post refused by a closing
// server restarts it (bounded: a server closes only after HG_OPT_SERVER_IDLE_US with nothing posted).
int server_render(hg_ctx* c, const HgKernelParams& kp, int32_t n_frames) {
    for (int32_t f = 0; f < n_frames; ++f) {
        const int32_t fc = c->params.frameCount + f;
        for (int attempt = 0;; ++attempt) {
            if (c->sv.running && !server_continues(c, fc))
                if (int rc = server_stop(c)) return rc;
            if (!c->sv.running) {
                const int rc = server_start(c, kp, fc);
                if (rc == HG_E_UNSUPPORTED && f > 0) return fail(c, HG_E_HIP, "render server: restart failed");
                if (rc) return rc;
            }
            const int rc = server_commit(c);
            if (rc != HG_E_UNSUPPORTED) {
                if (rc) return rc;
                break;
            }
            if (attempt >= 64) return fail(c, HG_E_HIP, "render server: 64 fresh servers in a row refused a post");
        }
    }
    server_speculate(c);
    return HG_OK;
}

// The host runs ahead of the GPU: the render call before the previous one has not finished on the device.  Then the
// render server pays: it removes the drain at each frame's end.  A host that waits for every frame (a display at once,
// or one frame behind) never runs ahead; the server serves it when it traces ahead of the calls (server_chain).
bool host_ahead(hg_ctx* c) {
    const int k = int(c->calls & 1u);  // recorded by the call before last
    if (!c->call_done_valid[k]) return false;
    const hipError_t q = hipEventQuery(c->call_done[k]);
    (void)hipGetLastError();  // hipErrorNotReady is a status here
    return q == hipErrorNotReady;
}
// The call continues a chain of at least two calls (same parameters, FrameCount continuing) and the server may trace
// ahead of it (HG_OPT_SERVER_AHEAD, counters off): the frames the host waits for are then already in flight
bool server_chain(hg_ctx* c, int32_t n_frames) {
    hg_params q = c->params;
    q.frameCount = 0;
    const bool cont = c->chain_len > 0 && c->params.frameCount == c->chain_next &&
                      std::memcmp(&q, &c->chain_params, sizeof q) == 0;
    c->chain_len = cont ? c->chain_len + 1 : 1;
    c->chain_params = q;
    c->chain_next = c->params.frameCount + n_frames;
    return c->sv_ahead > 0 && !c->counters_on && c->chain_len >= 2;
}
// After a render call's work is queued: its completion event, for host_ahead
void note_call(hg_ctx* c) {
    const int k = int(c->calls & 1u);
    c->call_done_valid[k] = hipEventRecord(c->call_done[k], c->stream) == hipSuccess;
    c->calls++;
}

// One launch of n_frames frames from FrameCount = params.frameCount (which it advances when accumulating)
int render_now(hg_ctx* c, int32_t n_frames, int32_t accumulate) {
    if (!c->has_scene) return fail(c, HG_E_NOSCENE, "hg_upload_scene not called");
    if (!c->has_params) return fail(c, HG_E_INVALID, "hg_set_params not called");
    if (c->W <= 0) return fail(c, HG_E_NOTARGET, "hg_resize not called");
    if (n_frames < 0) return fail(c, HG_E_INVALID, "n_frames < 0");
    const hg_params& p = c->params;
    if (int32_t(p.screenParameters.x) != c->W || int32_t(p.screenParameters.y) != c->H)
        return fail(c, HG_E_INVALID, "screenParameters (%g,%g) != target %dx%d", p.screenParameters.x,
                    p.screenParameters.y, c->W, c->H);
    const int32_t ns = int32_t(p.bufferCounts.x), nm = int32_t(p.bufferCounts.y);
    if (ns < 0 || ns > c->n_spheres || nm < 0 || nm > c->n_meshes)
        return fail(c, HG_E_INVALID, "bufferCounts (%d,%d) exceed uploaded (%d,%d)", ns, nm, c->n_spheres, c->n_meshes);
    if (n_frames == 0) return HG_OK;
    if (int rc = set_device(c)) return rc;

    HgKernelParams kp{};
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 4; ++k) kp.cam[r * 4 + k] = p.camLocalToWorld.m[k * 4 + r];
    kp.W = p.screenParameters.x;
    kp.H = p.screenParameters.y;
    kp.Wu = uint32_t(p.screenParameters.x);
    kp.Hu = uint32_t(c->H);
    kp.vw = p.viewParameters.x;
    kp.vh = p.viewParameters.y;
    kp.near_ = p.viewParameters.z;
    kp.far_ = p.viewParameters.w;
    // tan(radians(focalConeAngle)) * ViewParameters.z (:998), once per launch with the shared spec
    kp.focal_disc_radius = hg_tanf(p.focalConeAngle * HG_DEG2RAD) * p.viewParameters.z;
    kp.psx = (p.viewParameters.x * 2.0f) / p.screenParameters.x;  // get_ray_jitter :986
    kp.psy = (p.viewParameters.y * 2.0f) / p.screenParameters.y;
    kp.filter_radius = p.filterRadius;
    kp.focal_dist = p.focalPlaneDistance;
    kp.spp = p.samplesPerPixel;
    kp.max_bounces = p.maxBounces;
    kp.max_diff = p.maxDiffuseBounces;
    kp.max_glossy = p.maxGlossyBounces;
    kp.max_trans = p.maxTransmissionBounces;
    kp.debug_mode = p.halogenDebugMode;
    kp.tri_range = p.triangleDebugDisplayRange;
    kp.box_range = p.boxDebugDisplayRange;
    kp.default_mip = p.defaultHDRIMipLevel;
    kp.use_cube = (p.useEnvironmentCubemap > 0 && c->cube_mips > 0) ? 1 : 0;
    kp.n_spheres = ns;
    kp.n_meshes = nm;
    kp.first_frame = accumulate ? p.frameCount : 1;
    kp.n_frames = n_frames;
    kp.accumulate = accumulate ? 1 : 0;
    kp.frame_split = 1;
    kp.tiles_x = c->tiles_x;
    kp.rank = c->rank;
    kp.n_ranks = c->n_ranks;
    kp.n_local_tiles = c->n_local_tiles;
    kp.stack_depth = c->stack_depth;
    kp.cube_size = c->cube_size;
    kp.cube_mips = c->cube_mips;
    std::memcpy(kp.cube_mip_offset, c->cube_mip_offset, sizeof kp.cube_mip_offset);
    kp.spheres = static_cast<const float4*>(c->spheres.p);
    kp.meshes = static_cast<const HgDevMesh*>(c->meshes.p);
    kp.materials = static_cast<const float4*>(c->materials.p);
    kp.nodes = static_cast<const float4*>(c->nodes.p);
    kp.leaves = static_cast<const uint2*>(c->leaves.p);
    kp.tris = static_cast<const float*>(c->tris.p);
    kp.normals = static_cast<const float4*>(c->normals.p);
    kp.cube = static_cast<const float4*>(c->cube.p);
    kp.acc = static_cast<float4*>(c->acc.p);
    kp.counters = static_cast<unsigned long long*>(c->counters_dev.p);
    if (!c->counters_on) kp.counters = nullptr;

    std::pair<hipEvent_t, hipEvent_t> ev;
    if (int rc = event_pair(c, ev)) return rc;
    HG_HIP(c, hipEventRecord(ev.first, c->stream));
    // HG_KERNEL_AUTO: the streaming kernel for deep BLAS or many meshes, where traversals are long or uneven and its
    // resumable traversal lets a lane move on without waiting for the wave's slowest one (C3; C2's 9 meshes: 4,080
    // vs 3,891 Mpaths/s, tools/sweep_r02_ai.txt); the regenerating kernel for a few shallow meshes, where shading
    // dominates (C5's 2 meshes: 10,407 vs 9,718).  (Round 1, before the item scheduling and the mesh records in LDS,
    // the streaming kernel lost C2 too, tools/sweeps/sweep35.txt.)
    const bool deep_blas = c->stack_depth > HG_DESCENT_DEEP + 2;
    const bool stream_auto = deep_blas || c->n_meshes >= HG_STREAM_MIN_MESHES;
    const int32_t kern = c->kernel == HG_KERNEL_AUTO ? (stream_auto ? HG_KERNEL_MEGA_STREAM : HG_KERNEL_MEGA_REGEN)
                                                     : c->kernel;
    // relaxed descent threshold: 3 for the regen / lockstep kernels, HG_STREAM_DESCENT_T for the streaming one
    kp.stream_deep = deep_blas ? 1u : 0u;
    kp.descent_t = c->descent_t >= 0 ? uint32_t(c->descent_t)
                   : !deep_blas      ? 0u
                   : kern == HG_KERNEL_MEGA_STREAM ? uint32_t(HG_STREAM_DESCENT_T)
                                                   : uint32_t(HG_DESCENT_T);
    {
        const bool regen = (kern == HG_KERNEL_MEGA_REGEN || kern == HG_KERNEL_MEGA_STREAM) && p.halogenDebugMode == 0 &&
                           kp.max_bounces <= HG_REGEN_MAX_BOUNCES && kp.spp < HG_REGEN_MAX_CHUNK;
        // default block (option 128): 64 for the regenerating kernel (one tile per workgroup schedules best,
        // tools/sweeps/sweep12.txt), 256 for the lockstep one
        // the regenerating / streaming kernels run one wave per workgroup (their LDS row layout assumes it)
        const int mblock = regen ? 64 : (c->block == 128 ? 256 : c->block);
        // Frame-parallel split: `split` waves share each tile, each tracing a chunk of the frames, so a launch has
        // about 6x (formerly 16x, 12x) as many waves as the GPU holds at once (short waves: small drain tail; a rank's 1/N share
        // of the tiles at N GPUs still fills the GPU); the per-frame colours are then blended in frame order
        // (bit-identical).  Measured (tools/sweeps/sweep16-17.txt): C3 1080p 1180 -> 1251 Mpaths/s at N=1, and one
        // rank's share at N=8 314 -> 1212.
        const bool stream_k = regen && kern == HG_KERNEL_MEGA_STREAM;
        const int64_t tiles = c->n_local_tiles;
        const int64_t units = tiles;  // work units: one tile per wave
        const int64_t resident = int64_t(c->n_cu) * 4 * (stream_k ? HG_STREAM_WAVES : HG_MEGA_WAVES);
        int split = 1;
        if (regen && n_frames > 1 && tiles > 0) {
            if (c->frame_split > 0) split = std::min(n_frames, int(c->frame_split));
            // about 6 launches' worth of wave slots: with the cost order and a tile's chunks on consecutive waves
            // (wave_unit), fewer, longer waves win: a rank's share at N=2 split 2 vs 4 -> 2,409 vs 2,308, N=8 8 vs 16
            // -> 2,440 vs 2,337, C2 / C5 2 vs 3 -> +1.5 / +2.7 %, C3 at N=1 stays unsplit (tools/sweeps/sweep82-83.txt;
            // the multiplier was 16, then 12 with the chunk-major cost order)
            else split = int(std::min<int64_t>(n_frames, (6 * resident + units - 1) / units));
            // a share that runs the queue form (HG_OPT_QUEUE_FILL, below): smaller units, about 24 per wave slot, so
            // the launch's end leaves little behind (emulated N = 8 share of C3: split 8 / 16 / 32 -> 2,708 / 2,861 /
            // 2,933 Mpaths/s; per-tile waves at split 8: 2,790)
            if (c->frame_split <= 0 && kern == HG_KERNEL_MEGA_STREAM && n_frames > HG_QUEUE_MAX_FRAMES &&
                c->queue_fill > 0 && units * n_frames < int64_t(c->queue_fill) * resident * 64)
                split = int(std::min<int64_t>(n_frames, (int64_t(HG_QUEUE_FILL_UNITS) * resident + units - 1) / units));
        }
        // the AQL dispatch packet's grid size is a 32-bit count of work-items: at most 2^26 - 1 waves of 64 lanes
        constexpr int64_t kMaxWaves = (int64_t(1) << 26) - 1;
        if (units > kMaxWaves) {
            c->free_events.push_back(ev);
            return fail(c, HG_E_UNSUPPORTED, "target too large: %lld work units", (long long)units);
        }
        if (units > 0) split = int(std::min<int64_t>(split, kMaxWaves / units));
        int chunk_max = HG_REGEN_MAX_CHUNK;
        // The streaming kernel (always) and the regenerating kernel (item scheduling or a frame split) store every
        // frame's colour and blend them into the accumulator in frame order afterwards (hg_blend_frames): such a launch
        // is traced on a trace stream and blended on the context stream (the trace pipeline, hg_ctx.h).
        const bool items_k = regen && (stream_k || HG_REGEN_ITEMS);
        const bool pipelined = regen && (items_k || split > 1);
        const size_t per_frame = size_t(tiles) * 64 * sizeof(float4);
        if (pipelined)
            chunk_max = int(std::max<size_t>(1, std::min<size_t>(size_t(chunk_max), kFrameColorCap / per_frame)));
        const int mgrid = int((units * split + mblock / 64 - 1) / (mblock / 64));
        kp.spill_stride = uint32_t(mgrid) * uint32_t(mblock);
        // stack entries beyond the LDS part: one column per thread (the streaming kernel's LDS part may be shorter)
        const uint32_t lds_part = std::min<uint32_t>(HG_MEGA_LDS_STACK, HG_STREAM_LDS_STACK);
        const size_t spill_bytes =
            kp.stack_depth > lds_part ? size_t(kp.spill_stride) * (kp.stack_depth - lds_part) * 4 : 0;
        if (spill_bytes && !pipelined) {
            if (int rc = ensure_quiet(c, c->spill, spill_bytes)) {
                c->free_events.push_back(ev);
                return rc;
            }
            kp.spill = static_cast<uint32_t*>(c->spill.p);
        }

        c->counters.last_kernel = uint64_t(regen ? kern : HG_KERNEL_MEGA);
        // the reference's one frame per call: posted to the render server (persistent trace waves)
        const bool chain = accumulate && server_chain(c, n_frames);
        if (c->server_on && stream_k && pipelined && accumulate && n_frames <= HG_QUEUE_MAX_FRAMES && tiles > 0 &&
            (c->server_on == 2 || host_ahead(c) || chain)) {
            const int rc = server_render(c, kp, n_frames);
            if (rc == HG_OK) {
                HG_HIP(c, hipEventRecord(ev.second, c->stream));
                note_call(c);
                c->pending.push_back(ev);
                c->counters.launches++;
                if (c->pending.size() + c->pending_trace.size() > 4096)
                    if (int r = drain_events(c)) return r;
                c->params.frameCount += n_frames;  // FrameCount++ per accumulated frame (RP:347)
                return HG_OK;
            }
            if (rc != HG_E_UNSUPPORTED) {
                c->free_events.push_back(ev);
                return rc;
            }
        } else if (c->sv.running) {  // another kind of launch needs the GPU's wave slots
            if (int rc = server_stop(c)) {
                c->free_events.push_back(ev);
                return rc;
            }
        }
        hipError_t e = hipSuccess;
        const bool ordered = pipelined && c->tile_order_on && tiles > 0;
        const size_t tb = size_t(tiles) * sizeof(uint32_t);
        if (pipelined) {
            // the trace streams' buffers, grown only while idle (the lanes beyond HG_TRACE_LANES_BIG trace short chunks only)
            // the streams beyond HG_TRACE_LANES_BIG only when this launch has a chunk of at most HG_QUEUE_MAX_FRAMES
            // frames (the first, the last, or all of them), the rotation below that takes them
            const int last_chunk = n_frames % chunk_max;
            const bool short_chunks = std::min(n_frames, chunk_max) <= HG_QUEUE_MAX_FRAMES ||
                                      (last_chunk != 0 && last_chunk <= HG_QUEUE_MAX_FRAMES);
            for (int li = 0; li < HG_TRACE_LANES; ++li) {
                hg_ctx::TraceLane& L = c->lanes[li];
                if (li >= HG_TRACE_LANES_BIG && !short_chunks) continue;
                const int fmax = std::min(n_frames, li < HG_TRACE_LANES_BIG ? chunk_max
                                                                             : std::min(chunk_max, HG_QUEUE_MAX_FRAMES));
                int rc = ensure_quiet(c, L.frame_color, per_frame * size_t(fmax));
                if (!rc && spill_bytes) rc = ensure_quiet(c, L.spill, spill_bytes);
                if (!rc && ordered) rc = ensure_quiet(c, L.tile_cost, 2 * tb);
                if (!rc && ordered) rc = ensure_quiet(c, L.tile_order, tb);
                // the sort's scratch and the queue heads are zeroed once, when allocated (each use leaves them zeroed)
                const size_t osb = hg_order_scratch_bytes(uint32_t(tiles));
                if (!rc && ordered && L.order_scratch.bytes < osb) {
                    rc = ensure_quiet(c, L.order_scratch, osb);
                    if (!rc && hipMemsetAsync(L.order_scratch.p, 0, L.order_scratch.bytes, L.stream) != hipSuccess)
                        rc = fail(c, HG_E_HIP, "hipMemsetAsync(order scratch) failed");
                }
                const size_t qbytes = HG_QUEUE_BYTES;
                if (!rc && stream_k && L.queue.bytes < qbytes) {
                    rc = ensure_quiet(c, L.queue, qbytes);
                    if (!rc && hipMemsetAsync(L.queue.p, 0, L.queue.bytes, L.stream) != hipSuccess)
                        rc = fail(c, HG_E_HIP, "hipMemsetAsync(queue) failed");
                }
                if (rc) {
                    c->free_events.push_back(ev);
                    return rc;
                }
            }
            HgKernelParams kc = kp;
            const uint32_t slots = uint32_t(c->n_cu) * 4u * HG_STREAM_WAVES;
            for (int done = 0; done < n_frames && e == hipSuccess;) {  // chunks at frame boundaries change nothing
                kc.n_frames = std::min(n_frames - done, chunk_max);
                // short chunks (the reference's one dispatch per frame) in turn on every trace stream, so that more
                // launches' tails overlap; long ones on the first HG_TRACE_LANES_BIG (a third 64-frame launch beside
                // two others cost C3 1.5 %)
                int li;
                if (kc.n_frames <= HG_QUEUE_MAX_FRAMES) {
                    li = -1;
                    if (c->lane_pick) {  // the first stream whose last trace and blend are done (its queue stays warm)
                        for (int j = 0; j < HG_TRACE_LANES && li < 0; ++j)
                            if (!c->lanes[j].blend_pending || hipEventQuery(c->lanes[j].blended) == hipSuccess) li = j;
                        (void)hipGetLastError();  // hipErrorNotReady is a status here
                    }
                    if (li < 0) {
                        li = c->next_lane;
                        c->next_lane = (c->next_lane + 1) % HG_TRACE_LANES;
                    }
                } else {
                    li = c->next_lane_big;
                    c->next_lane_big = (c->next_lane_big + 1) % HG_TRACE_LANES_BIG;
                }
                hg_ctx::TraceLane& L = c->lanes[li];
                kc.first_frame = accumulate ? kp.first_frame + done : 1;
                kc.frame_split = std::min(split, kc.n_frames);
                kc.frame_color = static_cast<float4*>(L.frame_color.p);
                kc.spill = spill_bytes ? static_cast<uint32_t*>(L.spill.p) : nullptr;
                // the persistent work-queue form for launches of few frames (the reference's one dispatch per frame),
                // and for a launch too small to fill the GPU with 64-frame tile waves (a rank's 1/N of the image at N
                // GPUs, HG_OPT_QUEUE_FILL): persistent waves pull (tile, frame chunk) units, so a wave's lanes drain
                // once per launch, not once per short wave.  A share's launch of many frames fills the GPU with split
                // tile waves instead (emulated N = 8 share of C3, 512 frames: queue 3,289, split tile waves 3,543)
                const bool fill = c->queue_fill > 0 &&
                                  tiles * int64_t(kc.n_frames) < int64_t(c->queue_fill) * int64_t(slots) * 64;
                kc.queue = stream_k && (kc.n_frames <= HG_QUEUE_MAX_FRAMES || fill) ? static_cast<uint32_t*>(L.queue.p)
                                                                                     : nullptr;
                // Persistent waves of a queue launch.  A launch's end costs each of its waves the time its last paths
                // take, with its lanes draining; fewer, longer-lived waves pay that less often.  So while two or more
                // other traces are in flight (which fill the slots), a launch takes slots / min(HG_QUEUE_WAVES_DIV,
                // traces in flight + 1); alone or beside one other (e.g. a caller that reads every frame back), all.
                kc.resident_waves = slots;
                if (kc.queue && HG_QUEUE_WAVES_DIV > 1) {
                    int busy = 0;
                    for (const hg_ctx::TraceLane& O : c->lanes)
                        if (&O != &L && O.blend_pending && hipEventQuery(O.traced) == hipErrorNotReady) ++busy;
                    (void)hipGetLastError();  // hipErrorNotReady is a status here, not an error for the launch check
                    if (busy >= 2) kc.resident_waves = slots / uint32_t(std::min(HG_QUEUE_WAVES_DIV, busy + 1));
                }
                // Streaming launches without the queue and without a frame split: each wave traces wave_units
                // consecutive tiles of the cost order, its lanes draining once per wave instead of once per tile
                // (UnitItems), while the launch keeps at least HG_WAVE_UNITS_ROUNDS waves per resident slot
                kc.wave_units = 1;
                // (whole tiles only: a wave's units are all 8 x 8, UnitItems)
                if (stream_k && !kc.queue && kc.frame_split == 1 && tiles > 0 && c->W % HG_TILE == 0 &&
                    c->H % HG_TILE == 0) {
                    const int64_t auto_wu = std::min<int64_t>(HG_WAVE_UNITS_MAX, tiles / (int64_t(HG_WAVE_UNITS_ROUNDS) * slots));
                    kc.wave_units = uint32_t(c->wave_units > 0 ? c->wave_units : std::max<int64_t>(1, auto_wu));
                }
                kc.tile_order = nullptr;
                kc.tile_cost = ordered ? static_cast<unsigned long long*>(L.tile_cost.p) : nullptr;
                // this stream's buffers are free once the blend of its previous chunk has read them
                if (L.blend_pending) e = hipStreamWaitEvent(L.stream, L.blended, 0);
                if (e == hipSuccess && done == 0) e = hipEventRecord(ev.first, L.stream);  // the launch starts here
                if (e == hipSuccess && ordered) {
                    // Cost order, per trace stream: the stream sorts its own costs into its own order buffer (the
                    // traces adding those costs and reading that order run on the same stream, so none is in flight
                    // during the sort), once HG_ORDER_MIN_FRAMES frames were traced on it since its last sort:
                    // 64-frame launches every time, the reference's 1-frame launches every 16th frame per stream.
                    if (L.tile_cost_valid &&
                        (!L.tile_order_valid || L.frames_since_order >= int64_t(HG_ORDER_MIN_FRAMES))) {
                        e = hg_launch_order_tiles(kc.tile_cost, static_cast<uint32_t*>(L.tile_order.p), uint32_t(tiles),
                                                  L.order_scratch.p,
                                                  static_cast<unsigned long long*>(c->counters_dev.p) + 18, L.stream);
                        L.tile_order_valid = e == hipSuccess;
                        L.frames_since_order = 0;
                    } else if (!L.tile_cost_valid) {
                        e = hipMemsetAsync(kc.tile_cost, 0, size_t(tiles) * sizeof(unsigned long long), L.stream);
                        L.tile_order_valid = false;
                        L.frames_since_order = 0;
                    }
                    if (L.tile_order_valid) kc.tile_order = static_cast<const uint32_t*>(L.tile_order.p);
                    L.tile_cost_valid = e == hipSuccess;
                    L.frames_since_order += kc.n_frames;
                }
                std::pair<hipEvent_t, hipEvent_t> tev{};
                if (e == hipSuccess && c->timing) {
                    if (int rc = event_pair(c, tev)) {
                        c->free_events.push_back(ev);
                        return rc;
                    }
                    e = hipEventRecord(tev.first, L.stream);
                }
                if (e == hipSuccess)
                    e = stream_k ? hg_launch_mega_stream(kc, mblock, c->counters_on != 0, L.stream)
                                 : hg_launch_mega_regen(kc, mblock, c->counters_on != 0, L.stream);
                if (c->timing && tev.first) {  // a pair goes to drain_events only with both ends recorded
                    if (e == hipSuccess) e = hipEventRecord(tev.second, L.stream);
                    if (e == hipSuccess) c->pending_trace.push_back(tev);
                    else c->free_events.push_back(tev);
                }
                if (e == hipSuccess) e = hipEventRecord(L.traced, L.stream);
                if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, L.traced, 0);
                if (e == hipSuccess)  // in frame order, on the context stream
                    e = hg_launch_blend_frames(kc, static_cast<const uint32_t*>(c->lost.p), c->stream);
                if (e == hipSuccess) e = hipEventRecord(L.blended, c->stream);
                L.blend_pending = e == hipSuccess;
                done += kc.n_frames;
            }
            if (e != hipSuccess)  // a sort or a queue launch that failed part way may have left its words non-zero
                for (hg_ctx::TraceLane& L : c->lanes) {
                    if (L.queue.p) (void)hipMemsetAsync(L.queue.p, 0, L.queue.bytes, L.stream);
                    if (L.order_scratch.p) (void)hipMemsetAsync(L.order_scratch.p, 0, L.order_scratch.bytes, L.stream);
                    L.tile_cost_valid = L.tile_order_valid = false;
                }
        } else if (regen) {  // a regenerating launch that blends in the kernel (make noitems): on the context stream
            HgKernelParams kc = kp;
            for (int done = 0; done < n_frames && e == hipSuccess;) {
                kc.n_frames = std::min(n_frames - done, chunk_max);
                kc.first_frame = accumulate ? kp.first_frame + done : 1;
                kc.frame_split = std::min(split, kc.n_frames);
                e = hg_launch_mega_regen(kc, mblock, c->counters_on != 0, c->stream);
                done += kc.n_frames;
            }
        } else {
            e = hg_launch_mega(kp, mblock, c->counters_on != 0, c->stream);
        }
        if (e != hipSuccess) {
            c->free_events.push_back(ev);
            return fail(c, HG_E_HIP, "megakernel launch failed: %s", hipGetErrorString(e));
        }
    }
    HG_HIP(c, hipEventRecord(ev.second, c->stream));
    note_call(c);
    c->pending.push_back(ev);
    c->counters.launches++;
    if (c->pending.size() + c->pending_trace.size() > 4096) {
        if (int rc = drain_events(c)) return rc;
    }
    if (accumulate) c->params.frameCount += n_frames;  // FrameCount++ per accumulated frame (RP:347)
    return HG_OK;
}

}  // namespace

bool hg_ctx_lost(hg_ctx* c) {
    server_note_lost(c);
    return c->acc_lost;
}

int hg_ctx_flush(hg_ctx* c) {
    if (!c || c->pending_frames == 0) return HG_OK;
    const int32_t n = c->pending_frames, acc = c->pending_acc;
    c->pending_frames = 0;
    return render_now(c, n, acc);
}

// The accumulator (this rank's tiles, tile-major) as a row-major image in a display format (hg_pack.h); pixels of
// other ranks' tiles are 0.  One thread per pixel: the stores are contiguous (16 / 8 / 4 B per pixel), the loads are 8
// consecutive float4 per tile row.  64-thread workgroups (see launch_untile).
template <int kFmt, bool kRows>
__global__ __launch_bounds__(64) void hg_untile_image(void* __restrict__ image, const float4* __restrict__ acc,
                                                       int32_t W, int32_t H, int32_t tiles_x, int32_t rank,
                                                       int32_t n_ranks) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= uint32_t(W) * uint32_t(H)) return;
    float4 v;
    if constexpr (kRows) {  // the source is already a row-major image (the multi-GPU gather's assembled image)
        v = acc[i];
    } else {
        const HgPixelSource s = hg_pixel_source(i % uint32_t(W), i / uint32_t(W), uint32_t(tiles_x), uint32_t(n_ranks));
        v = s.rank == uint32_t(rank) ? acc[size_t(s.local_tile) * 64u + s.lane] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if constexpr (kFmt == HG_DISPLAY_RGBA32F) {
        static_cast<float4*>(image)[i] = v;
    } else if constexpr (kFmt == HG_DISPLAY_RGBA16F) {
        uint32_t h[2];
        hg_pack_rgba16f(v.x, v.y, v.z, v.w, h);
        static_cast<uint2*>(image)[i] = make_uint2(h[0], h[1]);
    } else {
        static_cast<uint32_t*>(image)[i] = hg_pack_r11g11b10(v.x, v.y, v.z);
    }
}

namespace {

size_t display_bpp(int32_t format) {
    return format == HG_DISPLAY_RGBA32F ? 16 : format == HG_DISPLAY_RGBA16F ? 8 : format == HG_DISPLAY_R11G11B10F ? 4 : 0;
}

template <bool kRows>
void launch_untile(hg_ctx* c, void* dst, int32_t format, const float4* src) {
    // one-wave workgroups with few registers: a display readback's untile runs beside the persistent trace waves of the
    // next frames (which hold most wave slots), as the lean blend does, instead of waiting for a CU to drain
    const size_t pixels = size_t(c->W) * size_t(c->H);
    const dim3 g(uint32_t((pixels + 63) / 64)), b(64);
    if (format == HG_DISPLAY_RGBA16F)
        hipLaunchKernelGGL((hg_untile_image<HG_DISPLAY_RGBA16F, kRows>), g, b, 0, c->stream, dst, src, c->W, c->H,
                           c->tiles_x, c->rank, c->n_ranks);
    else if (format == HG_DISPLAY_R11G11B10F)
        hipLaunchKernelGGL((hg_untile_image<HG_DISPLAY_R11G11B10F, kRows>), g, b, 0, c->stream, dst, src, c->W, c->H,
                           c->tiles_x, c->rank, c->n_ranks);
    else
        hipLaunchKernelGGL((hg_untile_image<HG_DISPLAY_RGBA32F, kRows>), g, b, 0, c->stream, dst, src, c->W, c->H,
                           c->tiles_x, c->rank, c->n_ranks);
}

// Enqueue on the context stream: the accumulator untiled (or, with `rows`, a row-major float4 image of the target's
// size converted) into `target` (c->image unless given; grown as needed) in `format`.  Returns its size in bytes.
int untile_async(hg_ctx* c, size_t* bytes, int32_t format = HG_DISPLAY_RGBA32F, const float4* rows = nullptr,
                 DevBuf* target = nullptr) {
    DevBuf& img = target ? *target : c->image;
    const size_t pixels = size_t(c->W) * size_t(c->H);
    *bytes = pixels * display_bpp(format);
    if (img.bytes < *bytes) {  // everything that might read the old image is ordered before on the context stream
        HG_HIP(c, hipStreamSynchronize(c->stream));
        if (int rc = ensure(c, img, *bytes)) return rc;
    }
    if (rows) launch_untile<true>(c, img.p, format, rows);
    else launch_untile<false>(c, img.p, format, static_cast<const float4*>(c->acc.p));
    HG_HIP(c, hipGetLastError());
    return HG_OK;
}

}  // namespace

// The display readback of hg_readback_begin_format, from the accumulator (rows == nullptr) or from a row-major float4
// image of the target's size on the context's device (the comm's assembled image, hg_comm_readback_begin)
int hg_ctx_display_begin(hg_ctx* c, const void* rows, int32_t format) {
    if (int rc = hg_ctx_flush(c)) return rc;
    if (c->W <= 0) return fail(c, HG_E_NOTARGET, "hg_resize not called");
    if (!display_bpp(format)) return fail(c, HG_E_INVALID, "unknown display format %d", format);
    if (c->rb_pending >= c->rb_depth)
        return fail(c, HG_E_INVALID, "%d readbacks outstanding (HG_OPT_READBACK_DEPTH): call hg_readback_end first",
                    c->rb_pending);
    if (int rc = set_device(c)) return rc;
    const int k = c->rb_next;  // not outstanding: at most rb_depth are, and k is the slot after the newest
    // HG_OPT_READBACK_STREAM 2 (zero copy): the untile kernel writes the display image straight into the slot's pinned
    // host image (mapped, fine-grained: its stores cross PCIe as they retire), no copy; the copy event is recorded
    // after the kernel on the context stream
    if (c->rb_side == 2) {
        const size_t bytes = size_t(c->W) * size_t(c->H) * display_bpp(format);
        if (c->image_host_cap[k] < bytes || !c->image_host_mapped[k]) {
            if (c->image_host[k]) {
                HG_HIP(c, hipEventSynchronize(c->image_copied[k]));  // (its last copy was ended: returns at once)
                HG_HIP(c, hipHostFree(c->image_host[k]));
            }
            c->image_host[k] = nullptr;
            c->image_host_cap[k] = 0;
            hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&c->image_host[k]), bytes,
                                         hipHostMallocMapped | hipHostMallocCoherent);
            if (e != hipSuccess) return fail(c, HG_E_NOMEM, "hipHostMalloc(%zu, mapped) failed: %s", bytes, hipGetErrorString(e));
            c->image_host_cap[k] = bytes;
            c->image_host_mapped[k] = true;
            if (!c->image_copied[k]) HG_HIP(c, hipEventCreateWithFlags(&c->image_copied[k], hipEventDisableTiming));
        }
        void* dptr = nullptr;
        HG_HIP(c, hipHostGetDevicePointer(&dptr, c->image_host[k], 0));
        if (rows) launch_untile<true>(c, dptr, format, static_cast<const float4*>(rows));
        else launch_untile<false>(c, dptr, format, static_cast<const float4*>(c->acc.p));
        HG_HIP(c, hipGetLastError());
        HG_HIP(c, hipEventRecord(c->image_copied[k], c->stream));
        c->image_host_bytes[k] = bytes;
        c->image_host_format[k] = format;
        c->rb_next = (k + 1) % c->rb_depth;
        c->rb_pending++;
        return HG_OK;
    }
    // HG_OPT_READBACK_STREAM 1: the slot's own device image, copied on the side stream, so the context stream (the next
    // frames' blends) does not wait for the copy; 0: c->image, copied on the context stream
    const bool side = c->rb_side != 0;
    if (side && !c->rb_stream) {
        // the copy stream on a hardware queue of its own (a plain stream shares one with a trace lane and waits behind
        // its traces: depth 2 1,285 -> 1,642 Mpaths/s, sweep_r04_rbq)
        HG_HIP(c, create_lane_stream(c, HG_TRACE_LANES, &c->rb_stream));
        for (int j = 0; j < HG_READBACK_MAX; ++j)
            HG_HIP(c, hipEventCreateWithFlags(&c->rb_untiled[j], hipEventDisableTiming));
    }
    size_t bytes = 0;
    DevBuf* dimg = side ? &c->rb_image[k] : &c->image;
    if (int rc = untile_async(c, &bytes, format, static_cast<const float4*>(rows), dimg)) return rc;
    if (c->image_host_cap[k] < bytes) {
        if (c->image_host[k]) {
            HG_HIP(c, hipEventSynchronize(c->image_copied[k]));  // (its last copy was ended, so this returns at once)
            HG_HIP(c, hipHostFree(c->image_host[k]));
        }
        c->image_host[k] = nullptr;
        c->image_host_cap[k] = 0;
        c->image_host_mapped[k] = false;
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&c->image_host[k]), bytes, 0);
        if (e != hipSuccess) return fail(c, HG_E_NOMEM, "hipHostMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
        c->image_host_cap[k] = bytes;
        if (!c->image_copied[k]) HG_HIP(c, hipEventCreateWithFlags(&c->image_copied[k], hipEventDisableTiming));
    }
    if (side) {
        HG_HIP(c, hipEventRecord(c->rb_untiled[k], c->stream));
        HG_HIP(c, hipStreamWaitEvent(c->rb_stream, c->rb_untiled[k], 0));
        HG_HIP(c, hipMemcpyAsync(c->image_host[k], dimg->p, bytes, hipMemcpyDeviceToHost, c->rb_stream));
        HG_HIP(c, hipEventRecord(c->image_copied[k], c->rb_stream));
    } else {
        HG_HIP(c, hipMemcpyAsync(c->image_host[k], dimg->p, bytes, hipMemcpyDeviceToHost, c->stream));
        HG_HIP(c, hipEventRecord(c->image_copied[k], c->stream));
    }
    c->image_host_bytes[k] = bytes;
    c->image_host_format[k] = format;
    c->rb_next = (k + 1) % c->rb_depth;
    c->rb_pending++;
    return HG_OK;
}

// The copy event of the oldest outstanding display readback (nullptr when none is outstanding)
hipEvent_t hg_ctx_display_oldest(const hg_ctx* c) {
    if (c->rb_pending <= 0) return nullptr;
    return c->image_copied[(c->rb_next - c->rb_pending + c->rb_depth) % c->rb_depth];
}

extern "C" {

int hg_readback_begin_format(hg_ctx* c, int32_t format) {
    if (!c) return HG_E_INVALID;
    return hg_ctx_display_begin(c, nullptr, format);
}

int hg_readback_begin(hg_ctx* c) { return hg_readback_begin_format(c, HG_DISPLAY_RGBA32F); }

int hg_readback_end_data(hg_ctx* c, const void** data, size_t* n_bytes, int32_t* format) {
    if (!c || !data) return HG_E_INVALID;
    if (c->rb_pending <= 0) return fail(c, HG_E_INVALID, "no readback outstanding: call hg_readback_begin first");
    if (int rc = set_device(c)) return rc;
    const int k = (c->rb_next - c->rb_pending + c->rb_depth) % c->rb_depth;  // the oldest begun
    HG_HIP(c, hipEventSynchronize(c->image_copied[k]));
    c->rb_pending--;
    *data = c->image_host[k];
    if (n_bytes) *n_bytes = c->image_host_bytes[k];
    if (format) *format = c->image_host_format[k];
    return lost_check(c);  // (the image is handed out either way: the accumulation through the last frame blended)
}

int hg_readback_end(hg_ctx* c, const float** rgba, size_t* n_floats) {
    if (!c || !rgba) return HG_E_INVALID;
    if (c->rb_pending <= 0) return fail(c, HG_E_INVALID, "no readback outstanding: call hg_readback_begin first");
    const int k = (c->rb_next - c->rb_pending + c->rb_depth) % c->rb_depth;
    if (c->image_host_format[k] != HG_DISPLAY_RGBA32F)
        return fail(c, HG_E_INVALID, "the oldest readback is in display format %d: use hg_readback_end_data",
                    c->image_host_format[k]);
    const void* data = nullptr;
    size_t bytes = 0;
    if (int rc = hg_readback_end_data(c, &data, &bytes, nullptr)) return rc;
    *rgba = static_cast<const float*>(data);
    if (n_floats) *n_floats = bytes / sizeof(float);
    return HG_OK;
}

int hg_pack_display(const float* rgba, size_t n_pixels, int32_t format, void* out) {
    if ((n_pixels && (!rgba || !out)) || !display_bpp(format)) return HG_E_INVALID;
    for (size_t i = 0; i < n_pixels; ++i) {
        const float* v = rgba + 4 * i;
        if (format == HG_DISPLAY_RGBA32F) {
            std::memcpy(static_cast<float*>(out) + 4 * i, v, 16);
        } else if (format == HG_DISPLAY_RGBA16F) {
            hg_pack_rgba16f(v[0], v[1], v[2], v[3], static_cast<uint32_t*>(out) + 2 * i);
        } else {
            static_cast<uint32_t*>(out)[i] = hg_pack_r11g11b10(v[0], v[1], v[2]);
        }
    }
    return HG_OK;
}

namespace {
// Frames of consecutive calls held for one launch (HG_OPT_COALESCE).  A rank's share of the image (N > 1) holds until
// its launch fills the GPU as one context's launch of the whole image does (HG_SHARE_HOLD_ROUNDS): a 1/8 share's
// 64-frame launch has 4,050 tiles for 5,120 wave slots, and its tail is as long as a full launch's.
int32_t hold_window(const hg_ctx* c) {
    int64_t w = c->coalesce;
    if (w > 1 && c->n_ranks > 1 && c->n_local_tiles > 0) {
        const int64_t slots = int64_t(c->n_cu) * 4 * HG_STREAM_WAVES;
        const int64_t share = (int64_t(HG_SHARE_HOLD_ROUNDS) * slots * 64 + c->n_local_tiles - 1) / c->n_local_tiles;
        w = std::max(w, std::min<int64_t>(share, HG_SHARE_HOLD_MAX));
    }
    return int32_t(w);
}
}  // namespace

int hg_render(hg_ctx* c, int32_t n_frames, int32_t accumulate) {
    if (!c) return HG_E_INVALID;
    if (int rc = render_check(c, n_frames)) return rc;
    if (int rc = lost_check(c)) return rc;
    if (n_frames == 0) return HG_OK;
    accumulate = accumulate ? 1 : 0;
    if (c->pending_frames > 0 && (accumulate != c->pending_acc || int64_t(c->pending_frames) + n_frames > INT32_MAX))
        if (int rc = hg_ctx_flush(c)) return rc;
    if (c->coalesce <= 1 && c->pending_frames == 0) return render_now(c, n_frames, accumulate);
    // held: the frames follow the held ones (FrameCount advances at the launch; nothing reads it before, every other
    // entry point flushes first)
    c->pending_acc = accumulate;
    c->pending_frames += n_frames;
    return c->pending_frames >= hold_window(c) ? hg_ctx_flush(c) : HG_OK;
}

int hg_synchronize(hg_ctx* c) {
    if (!c) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (int rc = set_device(c)) return rc;
    if (int rc = quiesce(c)) return rc;
    if (int rc = drain_events(c)) return rc;
    return lost_check(c);
}

int32_t hg_local_tile_count(const hg_ctx* c) { return c ? c->n_local_tiles : 0; }

int hg_readback(hg_ctx* c, float* rgba, size_t n_floats) {
    if (!c || !rgba) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (c->W <= 0) return fail(c, HG_E_NOTARGET, "hg_resize not called");
    if (n_floats < size_t(c->W) * size_t(c->H) * 4) return fail(c, HG_E_INVALID, "readback buffer too small");
    if (int rc = set_device(c)) return rc;
    if (c->n_ranks == 1) {  // the whole image: untiled on the device, one copy into the caller's memory
        size_t bytes = 0;
        if (int rc = untile_async(c, &bytes)) return rc;
        HG_HIP(c, hipMemcpyAsync(rgba, c->image.p, bytes, hipMemcpyDeviceToHost, c->stream));
        HG_HIP(c, hipStreamSynchronize(c->stream));
        if (int rc = drain_events(c)) return rc;
        return lost_check(c);  // (the image is written either way: the accumulation through the last frame blended)
    }
    // this rank's pixels only (the others are left untouched): the tiles are repacked on the host
    std::vector<float4> tiles(size_t(c->n_local_tiles) * 64);
    if (!tiles.empty())
        HG_HIP(c, hipMemcpyAsync(tiles.data(), c->acc.p, tiles.size() * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    HG_HIP(c, hipStreamSynchronize(c->stream));
    if (int rc = drain_events(c)) return rc;
    for (int32_t lt = 0; lt < c->n_local_tiles; ++lt) {
        const int64_t gt = int64_t(c->rank) + int64_t(lt) * c->n_ranks;
        const int tx = int(gt % c->tiles_x), ty = int(gt / c->tiles_x);
        for (int l = 0; l < 64; ++l) {
            const int x = tx * HG_TILE + (l & 7), y = ty * HG_TILE + (l >> 3);
            if (x >= c->W || y >= c->H) continue;
            const float4 v = tiles[size_t(lt) * 64 + l];
            float* d = rgba + (size_t(y) * c->W + x) * 4;
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
    }
    return lost_check(c);
}

int hg_set_accumulation(hg_ctx* c, const float* rgba, size_t n_floats, int32_t frame_count) {
    if (!c || !rgba) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (c->W <= 0) return fail(c, HG_E_NOTARGET, "hg_resize not called");
    if (n_floats < size_t(c->W) * size_t(c->H) * 4) return fail(c, HG_E_INVALID, "accumulation image too small");
    if (frame_count < 1) return fail(c, HG_E_INVALID, "frame_count must be >= 1 (FrameCount starts at 1, RP:152)");
    if (int rc = set_device(c)) return rc;
    // the tile-major repack of hg_readback, inverted; slots of an edge tile outside the image hold 0, as after a clear
    std::vector<float4> tiles(size_t(c->n_local_tiles) * 64, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (int32_t lt = 0; lt < c->n_local_tiles; ++lt) {
        const int64_t gt = int64_t(c->rank) + int64_t(lt) * c->n_ranks;
        const int tx = int(gt % c->tiles_x), ty = int(gt / c->tiles_x);
        for (int l = 0; l < 64; ++l) {
            const int x = tx * HG_TILE + (l & 7), y = ty * HG_TILE + (l >> 3);
            if (x >= c->W || y >= c->H) continue;
            const float* s = rgba + (size_t(y) * c->W + x) * 4;
            tiles[size_t(lt) * 64 + l] = make_float4(s[0], s[1], s[2], s[3]);
        }
    }
    if (!tiles.empty())
        HG_HIP(c, hipMemcpyAsync(c->acc.p, tiles.data(), tiles.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    if (int rc = reset_lost(c)) return rc;
    HG_HIP(c, hipStreamSynchronize(c->stream));  // the staging vector dies at return
    c->params.frameCount = frame_count;
    return drain_events(c);
}

int hg_copy_tiles_device(hg_ctx* c, void* dst, size_t n_bytes) {
    if (!c || !dst) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    const size_t need = size_t(c->n_local_tiles) * 64 * sizeof(float4);
    if (n_bytes < need) return fail(c, HG_E_INVALID, "destination too small (%zu < %zu)", n_bytes, need);
    if (int rc = set_device(c)) return rc;
    HG_HIP(c, hipStreamSynchronize(c->stream));  // every render kernel retired before the copy engine reads acc
    if (need) HG_HIP(c, hipMemcpyAsync(dst, c->acc.p, need, hipMemcpyDeviceToDevice, c->stream));
    HG_HIP(c, hipStreamSynchronize(c->stream));
    if (int rc = drain_events(c)) return rc;
    return lost_check(c);
}

int hg_get_counters(const hg_ctx* cc, hg_counters* out) {
    hg_ctx* c = const_cast<hg_ctx*>(cc);
    if (!c || !out) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (int rc = set_device(c)) return rc;
    if (int rc = server_stop(c)) return rc;  // (its waves add their counts when they leave)
    HG_HIP(c, hipStreamSynchronize(c->stream));
    if (int rc = drain_events(c)) return rc;
    unsigned long long v[32];
    HG_HIP(c, hipMemcpy(v, c->counters_dev.p, sizeof v, hipMemcpyDeviceToHost));
    *out = c->counters;
    out->paths = v[0];
    out->rays = v[1];
    out->tri_tests = v[2];
    out->aabb_tests = v[3];
    out->mesh_visits = v[4];
    out->sphere_tests = v[5];
    out->hits = v[6];
    out->node_rounds = v[7];
    out->tri_rounds = v[8];
    out->trace_cycles = v[9];
    out->shade_cycles = v[10];
    for (int k = 0; k < 4; ++k) out->shade_detail[k] = v[11 + k];
    out->shade_rounds = v[15];
    out->primary_misses = v[16];
    out->exec_fallbacks = v[17];
    out->order_faults = v[18];
    out->scene_uploads = c->scene_uploads;
    out->scene_uploads_skipped = c->scene_uploads_skipped;
    out->scene_uploads_partial = c->scene_uploads_partial;
    out->scene_uploads_vouched = c->scene_uploads_vouched;
    out->server_launches = c->server_launches;
    out->server_frames = c->server_frames;
    server_note_lost(c);
    out->server_refused = c->server_refused;
    out->server_ahead = c->server_ahead_posts;
    out->frames_lost = c->frames_lost;
    return HG_OK;
}

int hg_reset_counters(hg_ctx* c) {
    if (!c) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (int rc = set_device(c)) return rc;
    if (int rc = server_stop(c)) return rc;
    HG_HIP(c, hipStreamSynchronize(c->stream));
    if (int rc = drain_events(c)) return rc;
    HG_HIP(c, hipMemset(c->counters_dev.p, 0, c->counters_dev.bytes));
    c->counters = hg_counters{};
    return HG_OK;
}

int64_t hg_selftest(hg_ctx* c, int32_t test, int64_t* tested) {
    if (!c) return HG_E_INVALID;
    if (int rc = set_device(c)) return rc;
    if (test == HG_SELFTEST_BUILD) {  // compile-time checks of this build (no device work)
        if (tested) *tested = 0;
        return (HG_CHECK_EXEC ? HG_BUILD_CHECK_EXEC : 0) | (HG_REGEN_ITEMS ? 0 : HG_BUILD_NO_REGEN_ITEMS);
    }
    if (test != HG_SELFTEST_RCP) return fail(c, HG_E_INVALID, "unknown self-test %d", test);
    const int64_t r = hg_selftest_rcp_all(tested);
    if (r < 0) return fail(c, HG_E_HIP, "self-test failed to run");
    return r;
}

int hg_set_option(hg_ctx* c, int32_t option, int32_t value) {
    if (!c) return HG_E_INVALID;
    if (int rc = hg_ctx_flush(c)) return rc;
    if (c->sv.running) {  // every option changes what the server's waves were launched with
        if (int rc = set_device(c)) return rc;
        if (int rc = server_stop(c)) return rc;
    }
    switch (option) {
        case HG_OPT_KERNEL:
            if (value == HG_KERNEL_WAVEFRONT || value == HG_KERNEL_MEGA_POOL)
                return fail(c, HG_E_UNSUPPORTED, "kernel variant %d was measured, rejected and removed (DESIGN.md section 10)",
                            value);
            if (value != HG_KERNEL_MEGA && value != HG_KERNEL_MEGA_REGEN && value != HG_KERNEL_MEGA_STREAM &&
                value != HG_KERNEL_AUTO)
                return fail(c, HG_E_INVALID, "unknown kernel variant %d", value);
            c->kernel = value;
            return HG_OK;
        case HG_OPT_BLOCK:
            if (value != 64 && value != 128 && value != 256) return fail(c, HG_E_INVALID, "block must be 64/128/256");
            c->block = value;
            return HG_OK;
        case HG_OPT_COUNTERS:
            c->counters_on = value ? 1 : 0;
            return HG_OK;
        case HG_OPT_TIMING:
            c->timing = value ? 1 : 0;
            return HG_OK;
        case HG_OPT_REFILL:  // the wavefront pipeline's dequeue threshold
            return fail(c, HG_E_UNSUPPORTED, "HG_OPT_REFILL: the wavefront pipeline was removed (DESIGN.md section 10)");
        case HG_OPT_DESCENT_T:
            if (value < -1 || value > 64) return fail(c, HG_E_INVALID, "descent threshold must be -1 (auto)..64");
            c->descent_t = value;
            return HG_OK;
        case HG_OPT_TILE_ORDER:
            c->tile_order_on = value ? 1 : 0;
            for (hg_ctx::TraceLane& L : c->lanes) L.tile_cost_valid = L.tile_order_valid = false;
            return HG_OK;
        case HG_OPT_COALESCE:
            if (value < 1 || value > 65535) return fail(c, HG_E_INVALID, "coalesce window must be 1..65535 frames");
            c->coalesce = value;
            return HG_OK;
        case HG_OPT_READBACK_DEPTH:
            if (value < 1 || value > HG_READBACK_MAX)
                return fail(c, HG_E_INVALID, "readback depth must be 1..%d", HG_READBACK_MAX);
            if (c->rb_pending) return fail(c, HG_E_INVALID, "readbacks outstanding: end them before changing the depth");
            c->rb_depth = value;
            c->rb_next = 0;
            return HG_OK;
        case HG_OPT_READBACK_STREAM:
            if (c->rb_pending) return fail(c, HG_E_INVALID, "readbacks outstanding: end them before changing the stream");
            if (value < 0 || value > 2) return fail(c, HG_E_INVALID, "HG_OPT_READBACK_STREAM %d: expected 0, 1 or 2", value);
            c->rb_side = value;
            return HG_OK;
        case HG_OPT_FRAME_SPLIT:
            if (value < 0 || value > 4096) return fail(c, HG_E_INVALID, "frame split must be 0 (auto)..4096");
            c->frame_split = value;
            return HG_OK;
        case HG_OPT_LANE_PICK:
            c->lane_pick = value ? 1 : 0;
            return HG_OK;
        case HG_OPT_SERVER:
            if (value < 0 || value > 2) return fail(c, HG_E_INVALID, "HG_OPT_SERVER %d: expected 0, 1 or 2", value);
            c->server_on = value;
            return HG_OK;
        case HG_OPT_QUEUE_FILL:
            if (value < 0 || value > 64) return fail(c, HG_E_INVALID, "queue fill threshold must be 0 (off)..64 rounds");
            c->queue_fill = value;
            return HG_OK;
        case HG_OPT_SERVER_AHEAD:
            if (value < 0 || value > HG_SV_RING - 2) return fail(c, HG_E_INVALID, "server ahead must be 0..%d", HG_SV_RING - 2);
            c->sv_ahead = value;
            return HG_OK;
        case HG_OPT_SERVER_IDLE_US:
            if (value < 0 || value > 40000000) return fail(c, HG_E_INVALID, "server idle time must be 0..40000000 us");
            c->sv.idle_us = value;
            return HG_OK;
        case HG_OPT_SERVER_GATE_US:
            c->sv.gate_us = value;  // (< 0: the default)
            return HG_OK;
        case HG_OPT_WAVE_UNITS:
            if (value < 0 || value > HG_WAVE_UNITS_LIMIT)
                return fail(c, HG_E_INVALID, "wave units must be 0 (auto)..%d", HG_WAVE_UNITS_LIMIT);
            c->wave_units = value;
            return HG_OK;
        default:
            return fail(c, HG_E_INVALID, "unknown option %d", option);
    }
}

}  // extern "C"
