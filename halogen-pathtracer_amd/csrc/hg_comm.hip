// hg_comm.hip — multi-GPU framebuffer gather behind the C-ABI (include/halogen_abi.h, hg_comm_*).
//
// The reference is single-GPU (HalogenRenderPass.Execute, RP:270-357, renders the whole target).  Its pixels are
// independent — a pixel's value depends only on the scene, the uniforms, its GLOBAL index and FrameCount
// (HalgoenCompute.compute:1033) — so each GPU renders the interleaved 8x8 tiles t % N == rank (hg_set_tiling) and
// the only exchange is this gather of the accumulated tiles to the root, once per displayed image.
//
// Transport: RCCL point-to-point (ncclSend / ncclRecv; xGMI links between the GPUs of a node).
// Every RCCL call is enqueued on the rank context's own stream, so it is ordered after that context's renders on
// the device without a host wait, and the root's assembly kernel follows its receives on the same stream.  The
// root receives rank r's packed tiles into slab r of a staging buffer ([rank][max_local_tiles][64] float4) and one
// kernel (hg_assemble_image) writes the row-major image, reading its own tiles straight from its accumulator.
// hg_comm_init_all over contexts that share a device (a one-GPU rehearsal; RCCL refuses two ranks on one GPU) moves
// the slabs with device copies ordered by events instead.  Either way every byte the root reads was produced by a
// kernel or copy on a stream the root's stream waits on: no host-visible buffer, no foreign stream.
//
// Failure behaviour (SURVEY.md §5 "failure detection"): nothing here waits without a deadline.
//   - hg_comm_init_rank runs ncclCommInitRank on a helper thread and waits for it with the deadline: RCCL's own
//     "non-blocking" init (ncclConfig_t.blocking = 0) was measured to block in the calling thread while a peer is
//     missing.  An init abandoned at the deadline is aborted by its thread if it ever completes;
//   - every gather first agrees on the target size and tiling of all ranks (one 5-int ncclAllReduce, max of (v, -v)),
//     so a mismatched rank fails the gather on EVERY rank with the same text instead of leaving its peers blocked in
//     mismatched sends / receives; every ncclGroupStart is closed by its ncclGroupEnd on every path;
//   - waits (the agreement, hg_comm_synchronize, hg_comm_readback) poll the member streams and
//     ncclCommGetAsyncError; the deadline (hg_comm_set_timeout_ms, env HALOGEN_COMM_TIMEOUT_MS, default 120 s) starts
//     once this process's own renders ahead of the gather have retired, so only a missing or failed peer trips it.
//     On an RCCL error or a missed deadline every member communicator is aborted (ncclCommAbort) and the call returns
//     HG_E_COMM with text; the comm stays unusable (HG_E_COMM) until destroyed.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "halogen_abi.h"
#include "hg_ctx.h"
#include "hg_layout.h"
#include "hg_tiling.h"

namespace {
constexpr int kAgreeInts = 6;  // W, H, -W, -H, bad tiling, lost frame (max-reduced: equal on every rank iff max == -max(-v))
}

struct hg_comm {
    int32_t n_ranks = 0;
    int32_t transport = HG_COMM_RCCL;
    int64_t timeout_ms = 120000;
    bool aborted = false;
    std::string err;
    struct Member {
        hg_ctx* ctx = nullptr;
        int32_t rank = 0;
        ncclComm_t nccl = nullptr;  // RCCL transport
        hipEvent_t done = nullptr;  // peer transport: this rank's slab copy is complete (root: slabs free to write)
        hipEvent_t ready = nullptr;  // RCCL transport: recorded before this member's RCCL work (starts the deadline)
        int32_t* agree_dev = nullptr;   // RCCL transport: the agreement vector on the member's device
        int32_t* agree_host = nullptr;  // pinned: [0, 5) sent, [5, 10) received
    };
    std::vector<Member> members;  // the ranks driven by this process
    // root side (the member that last acted as root): staging slabs and the assembled image
    int32_t root = -1, W = 0, H = 0;
    hg_ctx* root_ctx = nullptr;
    int32_t buf_device = -1;  // device of slabs / image
    DevBuf slabs, image;
};

namespace {

int cfail(hg_comm* m, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (m) m->err = buf;
    return code;
}

#define HG_CHIP(comm, call)                                                                                  \
    do {                                                                                                     \
        hipError_t e_ = (call);                                                                              \
        if (e_ != hipSuccess) return cfail((comm), HG_E_HIP, "%s failed: %s", #call, hipGetErrorString(e_)); \
    } while (0)

int64_t env_timeout_ms() {
    const char* v = std::getenv("HALOGEN_COMM_TIMEOUT_MS");
    if (!v || !*v) return 120000;
    const long long t = std::atoll(v);
    return t > 0 ? int64_t(t) : 120000;
}

using Clock = std::chrono::steady_clock;

// HALOGEN_COMM_DEBUG=1: trace the communicator's waits on stderr (diagnostics of peer failures)
bool comm_debug() {
    static const bool on = [] {
        const char* v = std::getenv("HALOGEN_COMM_DEBUG");
        return v && *v && *v != '0';
    }();
    return on;
}
#define HG_CDBG(...)                                     \
    do {                                                 \
        if (comm_debug()) {                              \
            std::fprintf(stderr, "[hg_comm] " __VA_ARGS__); \
            std::fflush(stderr);                         \
        }                                                \
    } while (0)

// Abort every member communicator (RCCL's kernels of an aborted comm return) and make the comm unusable.
void abort_all(hg_comm* m) {
    for (auto& mb : m->members)
        if (mb.nccl) {
            HG_CDBG("ncclCommAbort rank %d\n", mb.rank);
            const ncclResult_t r = ncclCommAbort(mb.nccl);
            HG_CDBG("ncclCommAbort rank %d -> %s\n", mb.rank, ncclGetErrorString(r));
            mb.nccl = nullptr;
        }
    m->aborted = true;
}

// An RCCL error on any member communicator (remote failures surface here), or ncclSuccess / ncclInProgress
ncclResult_t async_state(hg_comm* m, int32_t* bad_rank) {
    ncclResult_t worst = ncclSuccess;
    for (auto& mb : m->members) {
        if (!mb.nccl) continue;
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = ncclCommGetAsyncError(mb.nccl, &st);
        if (r != ncclSuccess) st = r;
        if (st != ncclSuccess && st != ncclInProgress) {
            *bad_rank = mb.rank;
            return st;
        }
        if (st == ncclInProgress) worst = ncclInProgress;
    }
    return worst;
}

// Wait until every member communicator has finished its pending (non-blocking) operation: init, or a group call.
int wait_comms_ready(hg_comm* m, const char* what) {
    const auto deadline = Clock::now() + std::chrono::milliseconds(m->timeout_ms);
    HG_CDBG("%s: waiting up to %lld ms\n", what, (long long)m->timeout_ms);
    for (;;) {
        int32_t bad = -1;
        const ncclResult_t st = async_state(m, &bad);
        if (st == ncclSuccess) return HG_OK;
        if (st != ncclInProgress) {
            abort_all(m);
            return cfail(m, HG_E_COMM, "%s: RCCL error on rank %d: %s (communicator aborted)", what, bad,
                         ncclGetErrorString(st));
        }
        if (Clock::now() > deadline) {
            abort_all(m);
            return cfail(m, HG_E_COMM, "%s: not complete after %lld ms (a peer rank missing or stalled?); "
                                       "communicator aborted", what, (long long)m->timeout_ms);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// Wait for every member stream to drain.  The deadline starts once each member's `ready` event (recorded ahead of its
// RCCL work) has completed, i.e. once this process's own renders are done; RCCL errors are polled throughout.
// Wait until every member stream is idle (until_event == nullptr) or until `until_event` (an event on the root
// context's stream) has completed, bounded as hg_comm_synchronize documents.
int wait_streams(hg_comm* m, const char* what, hipEvent_t until_event = nullptr) {
    bool armed = m->transport != HG_COMM_RCCL;  // the peer transport has no remote party: plain deadline
    auto deadline = Clock::now() + std::chrono::milliseconds(m->timeout_ms);
    for (;;) {
        bool all_done = true, all_ready = true;
        if (until_event) {
            HG_CHIP(m, hipSetDevice(m->root_ctx->device));
            const hipError_t e = hipEventQuery(until_event);
            if (e == hipErrorNotReady) all_done = false;
            else if (e != hipSuccess) return cfail(m, HG_E_HIP, "%s: %s", what, hipGetErrorString(e));
        }
        for (auto& mb : m->members) {
            HG_CHIP(m, hipSetDevice(mb.ctx->device));
            const hipError_t e = until_event ? hipSuccess : hipStreamQuery(mb.ctx->stream);
            if (e == hipErrorNotReady) {
                all_done = false;
            } else if (e != hipSuccess) {
                return cfail(m, HG_E_HIP, "%s: stream of rank %d: %s", what, mb.rank, hipGetErrorString(e));
            }
            if (!armed && mb.ready) {
                const hipError_t r = hipEventQuery(mb.ready);
                if (r == hipErrorNotReady) all_ready = false;
                else if (r != hipSuccess)
                    return cfail(m, HG_E_HIP, "%s: event of rank %d: %s", what, mb.rank, hipGetErrorString(r));
            }
        }
        if (all_done) return HG_OK;
        if (!armed && all_ready) {
            armed = true;
            deadline = Clock::now() + std::chrono::milliseconds(m->timeout_ms);
        }
        int32_t bad = -1;
        const ncclResult_t st = async_state(m, &bad);
        if (st != ncclSuccess && st != ncclInProgress) {
            abort_all(m);
            return cfail(m, HG_E_COMM, "%s: RCCL error on rank %d: %s (communicator aborted)", what, bad,
                         ncclGetErrorString(st));
        }
        if (armed && Clock::now() > deadline) {
            if (m->transport == HG_COMM_RCCL) abort_all(m);
            return cfail(m, HG_E_COMM, "%s: not complete %lld ms after this process's renders retired (a peer rank "
                                       "missing or stalled?)%s", what, (long long)m->timeout_ms,
                         m->transport == HG_COMM_RCCL ? "; communicator aborted" : "");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

int ensure_buf(hg_comm* m, DevBuf& b, size_t bytes) {
    bytes = std::max<size_t>(bytes, 16);
    if (b.bytes >= bytes) return HG_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) return cfail(m, HG_E_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    b.bytes = bytes;
    return HG_OK;
}

// A member context's own view: tiled as (its rank, n_ranks) with a target.  0 = consistent.
int member_mismatch(const hg_comm* m, const hg_comm::Member& mb) {
    const hg_ctx* c = mb.ctx;
    return (c->n_ranks != m->n_ranks || c->rank != mb.rank || c->W <= 0) ? 1 : 0;
}

// Every member context must be tiled as (its rank, n_ranks) and hold a target of the same size (in-process check).
int check_member(hg_comm* m, const hg_comm::Member& mb, int32_t W, int32_t H) {
    const hg_ctx* c = mb.ctx;
    if (c->n_ranks != m->n_ranks || c->rank != mb.rank)
        return cfail(m, HG_E_COMM, "context of rank %d is tiled as %d/%d, not %d/%d", mb.rank, c->rank, c->n_ranks,
                     mb.rank, m->n_ranks);
    if (c->W <= 0) return cfail(m, HG_E_NOTARGET, "rank %d: hg_resize not called", mb.rank);
    if (c->W != W || c->H != H)
        return cfail(m, HG_E_COMM, "rank %d target %dx%d differs from %dx%d", mb.rank, c->W, c->H, W, H);
    return HG_OK;
}

// RCCL transport: every rank of the communicator contributes (W, H, -W, -H, bad, lost) and max-reduces; all ranks then
// hold the same verdict, so a mismatch, or an accumulation invalidated by a lost render-server frame on any rank
// (HG_E_FRAME_LOST), fails the gather everywhere before any send / receive is posted.
int agree_on_target(hg_comm* m, int32_t& W, int32_t& H) {
    for (auto& mb : m->members) {
        const hg_ctx* c = mb.ctx;
        int32_t* v = mb.agree_host;
        v[0] = c->W;
        v[1] = c->H;
        v[2] = -c->W;
        v[3] = -c->H;
        v[4] = member_mismatch(m, mb);
        v[5] = hg_ctx_lost(mb.ctx) ? 1 : 0;
        HG_CHIP(m, hipSetDevice(c->device));
        HG_CHIP(m, hipEventRecord(mb.ready, c->stream));
        HG_CHIP(m, hipMemcpyAsync(mb.agree_dev, v, kAgreeInts * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    }
    ncclResult_t gr = ncclGroupStart();
    if (gr != ncclSuccess) return cfail(m, HG_E_COMM, "ncclGroupStart failed: %s", ncclGetErrorString(gr));
    ncclResult_t first = ncclSuccess;
    for (auto& mb : m->members) {
        const ncclResult_t r =
            ncclAllReduce(mb.agree_dev, mb.agree_dev, kAgreeInts, ncclInt32, ncclMax, mb.nccl, mb.ctx->stream);
        if (r != ncclSuccess && r != ncclInProgress && first == ncclSuccess) first = r;
    }
    gr = ncclGroupEnd();  // always closes the group, also after a failed enqueue
    if (first != ncclSuccess) {
        abort_all(m);
        return cfail(m, HG_E_COMM, "ncclAllReduce (gather agreement) failed: %s", ncclGetErrorString(first));
    }
    if (gr == ncclInProgress) {
        if (int rc = wait_comms_ready(m, "gather agreement")) return rc;
    } else if (gr != ncclSuccess) {
        abort_all(m);
        return cfail(m, HG_E_COMM, "ncclGroupEnd (gather agreement) failed: %s", ncclGetErrorString(gr));
    }
    for (auto& mb : m->members) {
        HG_CHIP(m, hipSetDevice(mb.ctx->device));
        HG_CHIP(m, hipMemcpyAsync(mb.agree_host + kAgreeInts, mb.agree_dev, kAgreeInts * sizeof(int32_t),
                                  hipMemcpyDeviceToHost, mb.ctx->stream));
    }
    if (int rc = wait_streams(m, "gather agreement")) return rc;
    const int32_t* r = m->members.front().agree_host + kAgreeInts;
    if (r[4] != 0) {
        for (auto& mb : m->members)
            if (member_mismatch(m, mb))
                return cfail(m, HG_E_COMM, "context of rank %d is tiled as %d/%d (target %dx%d), not %d/%d", mb.rank,
                             mb.ctx->rank, mb.ctx->n_ranks, mb.ctx->W, mb.ctx->H, mb.rank, m->n_ranks);
        return cfail(m, HG_E_COMM, "a peer rank's context is not tiled for this communicator or has no target");
    }
    if (r[5] != 0)
        return cfail(m, HG_E_FRAME_LOST, "a rank's accumulation is invalid: a render server frame was lost there");
    if (r[0] != -r[2] || r[1] != -r[3])
        return cfail(m, HG_E_COMM, "ranks disagree on the target size (widths %d..%d, heights %d..%d)", -r[2], r[0],
                     -r[3], r[1]);
    W = r[0];
    H = r[1];
    return HG_OK;
}

// Release the staging buffers on the device that holds them, after that device's work on them has retired.
void free_staging(hg_comm* m) {
    if (m->buf_device >= 0 && (m->slabs.p || m->image.p)) {
        (void)hipSetDevice(m->buf_device);
        if (m->root_ctx) (void)hipStreamSynchronize(m->root_ctx->stream);
        (void)hipDeviceSynchronize();
        for (DevBuf* b : {&m->slabs, &m->image}) {
            if (b->p) (void)hipFree(b->p);
            *b = DevBuf{};
        }
    }
    m->buf_device = -1;
}

int alloc_member_rccl(hg_comm* m, hg_comm::Member& mb) {
    HG_CHIP(m, hipSetDevice(mb.ctx->device));
    HG_CHIP(m, hipEventCreateWithFlags(&mb.ready, hipEventDisableTiming));
    HG_CHIP(m, hipMalloc(reinterpret_cast<void**>(&mb.agree_dev), 64));
    HG_CHIP(m, hipHostMalloc(reinterpret_cast<void**>(&mb.agree_host), 2 * kAgreeInts * sizeof(int32_t), 0));
    return HG_OK;
}

}  // namespace

// Row-major image from the root's own accumulator (tiles of the root rank) and the received slabs (other ranks),
// through the mapping of hg_tiling.h.
__global__ __launch_bounds__(256) void hg_assemble_image(float4* __restrict__ image, const float4* __restrict__ own,
                                                         const float4* __restrict__ slabs, int32_t W, int32_t H,
                                                         int32_t tiles_x, int32_t n, int32_t root,
                                                         uint32_t slab_tiles) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= uint32_t(W) * uint32_t(H)) return;
    const HgPixelSource s = hg_pixel_source(i % uint32_t(W), i / uint32_t(W), uint32_t(tiles_x), uint32_t(n));
    image[i] = s.rank == uint32_t(root) ? own[size_t(s.local_tile) * 64u + s.lane] : slabs[hg_slab_index(s, slab_tiles)];
}

extern "C" {

int hg_comm_unique_id(uint8_t id[HG_COMM_ID_BYTES]) {
    static_assert(HG_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "id size");
    if (!id) return HG_E_INVALID;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return HG_E_COMM;
    std::memcpy(id, u.internal, HG_COMM_ID_BYTES);
    return HG_OK;
}

int hg_comm_init_rank(hg_ctx* ctx, int32_t n_ranks, const uint8_t id[HG_COMM_ID_BYTES], int32_t rank,
                      hg_comm** out) {
    if (!ctx || !id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks) return HG_E_INVALID;
    *out = nullptr;
    hg_comm* m = new hg_comm();
    m->n_ranks = n_ranks;
    m->transport = HG_COMM_RCCL;
    m->timeout_ms = env_timeout_ms();
    m->members.resize(1);
    hg_comm::Member& mb = m->members.front();
    mb.ctx = ctx;
    mb.rank = rank;
    ncclUniqueId u;
    std::memcpy(u.internal, id, HG_COMM_ID_BYTES);
    if (int rc = alloc_member_rccl(m, mb)) {
        ctx->err = m->err;
        hg_comm_destroy(m);
        return rc;
    }
    // The init blocks until every rank has joined: a helper thread makes the call and this one waits with the
    // deadline.  At the deadline the job is abandoned; its thread aborts the communicator if the init ever returns.
    struct InitJob {
        std::mutex mu;
        std::condition_variable cv;
        bool done = false, abandoned = false;
        ncclComm_t comm = nullptr;
        ncclResult_t r = ncclSuccess;
    };
    auto job = std::make_shared<InitJob>();
    const int dev = ctx->device;
    HG_CDBG("ncclCommInitRank rank %d of %d on a helper thread, deadline %lld ms\n", rank, n_ranks,
            (long long)m->timeout_ms);
    try {
        std::thread([job, n_ranks, u, rank, dev]() {
            ncclComm_t cm = nullptr;
            ncclResult_t r = hipSetDevice(dev) == hipSuccess ? ncclCommInitRank(&cm, n_ranks, u, rank)
                                                             : ncclUnhandledCudaError;
            std::lock_guard<std::mutex> lk(job->mu);
            if (job->abandoned) {
                if (cm) (void)ncclCommAbort(cm);
                return;
            }
            job->comm = cm;
            job->r = r;
            job->done = true;
            job->cv.notify_all();
        }).detach();
    } catch (const std::exception& ex) {
        ctx->err = std::string("hg_comm_init_rank: cannot start the init thread: ") + ex.what();
        hg_comm_destroy(m);
        return HG_E_COMM;
    }
    int rc = HG_OK;
    {
        std::unique_lock<std::mutex> lk(job->mu);
        if (!job->cv.wait_for(lk, std::chrono::milliseconds(m->timeout_ms), [&] { return job->done; })) {
            job->abandoned = true;
            rc = cfail(m, HG_E_COMM, "ncclCommInitRank: rank %d of %d: the other ranks did not all join within %lld ms "
                                     "(a peer missing or failed?); init abandoned", rank, n_ranks,
                       (long long)m->timeout_ms);
        } else if (job->r != ncclSuccess) {
            rc = cfail(m, HG_E_COMM, "ncclCommInitRank failed: %s", ncclGetErrorString(job->r));
            if (job->comm) (void)ncclCommAbort(job->comm);
        } else {
            mb.nccl = job->comm;
        }
    }
    HG_CDBG("ncclCommInitRank -> %d\n", rc);
    if (rc != HG_OK) {
        ctx->err = m->err;
        hg_comm_destroy(m);
        return rc;
    }
    *out = m;
    return HG_OK;
}

int hg_comm_init_all(hg_ctx* const* ctxs, int32_t n_ranks, hg_comm** out) {
    if (!ctxs || !out || n_ranks < 1) return HG_E_INVALID;
    *out = nullptr;
    std::vector<int> devs(static_cast<size_t>(n_ranks));
    for (int32_t r = 0; r < n_ranks; ++r) {
        if (!ctxs[r]) return HG_E_INVALID;
        devs[size_t(r)] = ctxs[r]->device;
    }
    std::vector<int> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    hg_comm* m = new hg_comm();
    m->n_ranks = n_ranks;
    m->transport = distinct ? HG_COMM_RCCL : HG_COMM_PEER;
    m->timeout_ms = env_timeout_ms();
    m->members.resize(size_t(n_ranks));
    std::vector<ncclComm_t> comms(size_t(n_ranks), nullptr);
    if (distinct) {
        const ncclResult_t r = ncclCommInitAll(comms.data(), n_ranks, devs.data());
        if (r != ncclSuccess) {
            ctxs[0]->err = std::string("ncclCommInitAll failed: ") + ncclGetErrorString(r);
            delete m;
            return HG_E_COMM;
        }
    }
    for (int32_t r = 0; r < n_ranks; ++r) {
        hg_comm::Member& mb = m->members[size_t(r)];
        mb.ctx = ctxs[r];
        mb.rank = r;
        mb.nccl = comms[size_t(r)];
        int rc = HG_OK;
        if (distinct) {
            rc = alloc_member_rccl(m, mb);
        } else if (hipSetDevice(mb.ctx->device) != hipSuccess ||
                   hipEventCreateWithFlags(&mb.done, hipEventDisableTiming) != hipSuccess) {
            rc = HG_E_HIP;
        }
        if (rc != HG_OK) {
            ctxs[0]->err = m->err.empty() ? "hg_comm_init_all: HIP setup failed" : m->err;
            hg_comm_destroy(m);
            return rc;
        }
    }
    *out = m;
    return HG_OK;
}

int hg_comm_set_timeout_ms(hg_comm* m, int64_t timeout_ms) {
    if (!m) return HG_E_INVALID;
    if (timeout_ms <= 0) return cfail(m, HG_E_INVALID, "timeout must be > 0 ms");
    m->timeout_ms = timeout_ms;
    return HG_OK;
}

int hg_comm_gather(hg_comm* m, int32_t root) {
    if (!m) return HG_E_INVALID;
    if (m->aborted) return cfail(m, HG_E_COMM, "communicator was aborted after an earlier failure");
    if (root < 0 || root >= m->n_ranks) return cfail(m, HG_E_INVALID, "root %d out of range", root);
    for (auto& mb : m->members)  // held hg_render frames are launched before the accumulators are read
        if (hg_ctx_flush(mb.ctx) != HG_OK) return cfail(m, HG_E_HIP, "rank %d: %s", mb.rank, mb.ctx->err.c_str());
    int32_t W = m->members.front().ctx->W, H = m->members.front().ctx->H;
    if (m->transport == HG_COMM_RCCL) {
        if (int rc = agree_on_target(m, W, H)) return rc;
    } else {
        for (const auto& mb : m->members)
            if (int rc = check_member(m, mb, W, H)) return rc;
        for (const auto& mb : m->members)
            if (hg_ctx_lost(mb.ctx))
                return cfail(m, HG_E_FRAME_LOST, "rank %d: its accumulation is invalid (a render server frame was lost)",
                             mb.rank);
    }
    const hg_ctx* c0 = m->members.front().ctx;
    const int32_t n = m->n_ranks;
    const int64_t total = int64_t(c0->tiles_x) * c0->tiles_y;
    const int64_t slab_tiles = hg_rank_tiles(total, 0, n);  // rank 0 holds the most tiles
    const size_t slab_floats = size_t(slab_tiles) * 64 * 4;
    hg_comm::Member* rootm = nullptr;
    for (auto& mb : m->members)
        if (mb.rank == root) rootm = &mb;
    if (rootm) {  // this process holds the root: staging slabs and the image on its device
        if (m->buf_device != rootm->ctx->device) free_staging(m);  // a root on another device: its own staging
        HG_CHIP(m, hipSetDevice(rootm->ctx->device));
        m->buf_device = rootm->ctx->device;
        if (int rc = ensure_buf(m, m->slabs, size_t(n) * slab_floats * sizeof(float))) return rc;
        if (int rc = ensure_buf(m, m->image, size_t(W) * size_t(H) * sizeof(float4))) return rc;
    }
    m->root = -1;  // valid again once the assembly is enqueued
    if (m->transport == HG_COMM_RCCL) {
        ncclResult_t gr = ncclGroupStart();
        if (gr != ncclSuccess) return cfail(m, HG_E_COMM, "ncclGroupStart failed: %s", ncclGetErrorString(gr));
        ncclResult_t first = ncclSuccess;
        const char* first_what = "";
        auto note = [&](ncclResult_t r, const char* what) {
            if (r != ncclSuccess && r != ncclInProgress && first == ncclSuccess) {
                first = r;
                first_what = what;
            }
        };
        for (auto& mb : m->members) {
            const size_t cnt = size_t(hg_rank_tiles(total, mb.rank, n)) * 64 * 4;
            if (mb.rank == root) {
                for (int32_t r = 0; r < n; ++r) {
                    const size_t rc = size_t(hg_rank_tiles(total, r, n)) * 64 * 4;
                    if (r == root || rc == 0) continue;
                    float* dst = static_cast<float*>(m->slabs.p) + size_t(r) * slab_floats;
                    note(ncclRecv(dst, rc, ncclFloat32, r, mb.nccl, mb.ctx->stream), "ncclRecv");
                }
            } else if (cnt) {
                note(ncclSend(mb.ctx->acc.p, cnt, ncclFloat32, root, mb.nccl, mb.ctx->stream), "ncclSend");
            }
        }
        gr = ncclGroupEnd();  // always closes the group, also after a failed enqueue
        if (first != ncclSuccess) {
            abort_all(m);
            return cfail(m, HG_E_COMM, "%s failed: %s (communicator aborted)", first_what, ncclGetErrorString(first));
        }
        if (gr == ncclInProgress) {
            if (int rc = wait_comms_ready(m, "gather send/recv group")) return rc;
        } else if (gr != ncclSuccess) {
            abort_all(m);
            return cfail(m, HG_E_COMM, "ncclGroupEnd failed: %s (communicator aborted)", ncclGetErrorString(gr));
        }
    } else {  // peer transport: every member is in this process and rootm is set
        // the slabs are free once the root's previous assembly has read them
        HG_CHIP(m, hipEventRecord(rootm->done, rootm->ctx->stream));
        for (auto& mb : m->members) {
            if (mb.rank == root) continue;
            HG_CHIP(m, hipSetDevice(mb.ctx->device));
            HG_CHIP(m, hipStreamWaitEvent(mb.ctx->stream, rootm->done, 0));
            const size_t bytes = size_t(hg_rank_tiles(total, mb.rank, n)) * 64 * sizeof(float4);
            if (bytes) {
                float* dst = static_cast<float*>(m->slabs.p) + size_t(mb.rank) * slab_floats;
                HG_CHIP(m, hipMemcpyPeerAsync(dst, rootm->ctx->device, mb.ctx->acc.p, mb.ctx->device, bytes,
                                              mb.ctx->stream));
            }
            HG_CHIP(m, hipEventRecord(mb.done, mb.ctx->stream));
            HG_CHIP(m, hipSetDevice(rootm->ctx->device));
            HG_CHIP(m, hipStreamWaitEvent(rootm->ctx->stream, mb.done, 0));
        }
    }
    if (rootm) {
        hg_ctx* rc = rootm->ctx;
        HG_CHIP(m, hipSetDevice(rc->device));
        const uint32_t px = uint32_t(W) * uint32_t(H);
        hipLaunchKernelGGL(hg_assemble_image, dim3((px + 255) / 256), dim3(256), 0, rc->stream,
                           static_cast<float4*>(m->image.p), static_cast<const float4*>(rc->acc.p),
                           static_cast<const float4*>(m->slabs.p), W, H, rc->tiles_x, n, root, uint32_t(slab_tiles));
        HG_CHIP(m, hipGetLastError());
        m->root = root;
        m->root_ctx = rc;
        m->W = W;
        m->H = H;
    }
    return HG_OK;
}

int hg_comm_synchronize(hg_comm* m) {
    if (!m) return HG_E_INVALID;
    if (m->aborted) return cfail(m, HG_E_COMM, "communicator was aborted after an earlier failure");
    return wait_streams(m, "hg_comm_synchronize");
}

int hg_comm_readback(hg_comm* m, float* rgba, size_t n_floats) {
    if (!m || !rgba) return HG_E_INVALID;
    if (m->aborted) return cfail(m, HG_E_COMM, "communicator was aborted after an earlier failure");
    if (m->root < 0 || !m->root_ctx) return cfail(m, HG_E_INVALID, "no gathered image in this process");
    if (n_floats < size_t(m->W) * size_t(m->H) * 4) return cfail(m, HG_E_INVALID, "readback buffer too small");
    if (int rc = wait_streams(m, "hg_comm_readback")) return rc;  // the receives, bounded by the deadline
    hg_ctx* rc = m->root_ctx;
    HG_CHIP(m, hipSetDevice(rc->device));
    HG_CHIP(m, hipMemcpyAsync(rgba, m->image.p, size_t(m->W) * size_t(m->H) * sizeof(float4), hipMemcpyDeviceToHost,
                              rc->stream));
    HG_CHIP(m, hipStreamSynchronize(rc->stream));
    for (const auto& mb : m->members)  // (a frame lost after the gather's agreement: the image is handed out, flagged)
        if (hg_ctx_lost(mb.ctx))
            return cfail(m, HG_E_FRAME_LOST, "rank %d: its accumulation is invalid (a render server frame was lost)",
                         mb.rank);
    return HG_OK;
}

// Pipelined display of the gathered image (the multi-GPU form of hg_readback_begin_format / hg_readback_end_data):
// enqueued on the root context's stream after the last gather's assembly, into that context's ring of pinned host
// images (HG_OPT_READBACK_DEPTH of the root context); the end waits for the oldest one with the deadline of
// hg_comm_synchronize, so a dead peer cannot hang the display.
int hg_comm_readback_begin(hg_comm* m, int32_t format) {
    if (!m) return HG_E_INVALID;
    if (m->aborted) return cfail(m, HG_E_COMM, "communicator was aborted after an earlier failure");
    if (m->root < 0 || !m->root_ctx) return cfail(m, HG_E_INVALID, "no gathered image in this process");
    hg_ctx* rc = m->root_ctx;
    if (rc->W != m->W || rc->H != m->H) return cfail(m, HG_E_INVALID, "the root context was resized after the gather");
    if (int e = hg_ctx_display_begin(rc, m->image.p, format)) return cfail(m, e, "%s", rc->err.c_str());
    return HG_OK;
}

int hg_comm_readback_end(hg_comm* m, const void** data, size_t* n_bytes, int32_t* format) {
    if (!m || !data) return HG_E_INVALID;
    if (m->aborted) return cfail(m, HG_E_COMM, "communicator was aborted after an earlier failure");
    if (!m->root_ctx) return cfail(m, HG_E_INVALID, "no gathered image in this process");
    hipEvent_t ev = hg_ctx_display_oldest(m->root_ctx);
    if (!ev) return cfail(m, HG_E_INVALID, "no readback outstanding: call hg_comm_readback_begin first");
    if (int rc = wait_streams(m, "hg_comm_readback_end", ev)) return rc;
    if (int e = hg_readback_end_data(m->root_ctx, data, n_bytes, format))
        return cfail(m, e, "%s", m->root_ctx->err.c_str());
    for (const auto& mb : m->members)
        if (hg_ctx_lost(mb.ctx))
            return cfail(m, HG_E_FRAME_LOST, "rank %d: its accumulation is invalid (a render server frame was lost)",
                         mb.rank);
    return HG_OK;
}

int hg_comm_transport(const hg_comm* m) { return m ? m->transport : HG_E_INVALID; }

const char* hg_comm_last_error(const hg_comm* m) { return m ? m->err.c_str() : "null communicator"; }

void hg_comm_destroy(hg_comm* m) {
    if (!m) return;
    for (auto& mb : m->members) {
        // after an abort a member stream may hold an RCCL kernel of the aborted comm: do not wait on it
        if (mb.ctx && !m->aborted) {
            (void)hipSetDevice(mb.ctx->device);
            (void)hipStreamSynchronize(mb.ctx->stream);
        }
        if (mb.nccl) (void)ncclCommDestroy(mb.nccl);
        if (mb.done) (void)hipEventDestroy(mb.done);
        if (mb.ready) (void)hipEventDestroy(mb.ready);
        if (mb.agree_dev) (void)hipFree(mb.agree_dev);
        if (mb.agree_host) (void)hipHostFree(mb.agree_host);
    }
    if (!m->aborted) free_staging(m);
    delete m;
}

// Host twin of hg_assemble_image over the [rank][slab_tiles][64] float4 layout (slab r = rank r's local tiles, the
// root's own included): the torch all_gather path (halogen/distributed.py) and the CPU tests use it.  No device work.
int hg_comm_assemble_host(const float* slabs, int64_t slab_tiles, int32_t width, int32_t height, int32_t n_ranks,
                          float* rgba, size_t n_floats) {
    if (!slabs || !rgba || width <= 0 || height <= 0 || n_ranks < 1) return HG_E_INVALID;
    const int64_t tiles_x = (width + HG_TILE - 1) / HG_TILE, tiles_y = (height + HG_TILE - 1) / HG_TILE;
    if (slab_tiles < hg_rank_tiles(tiles_x * tiles_y, 0, n_ranks)) return HG_E_INVALID;
    if (n_floats < size_t(width) * size_t(height) * 4) return HG_E_INVALID;
    for (int32_t y = 0; y < height; ++y)
        for (int32_t x = 0; x < width; ++x) {
            const HgPixelSource s = hg_pixel_source(uint32_t(x), uint32_t(y), uint32_t(tiles_x), uint32_t(n_ranks));
            std::memcpy(rgba + (size_t(y) * size_t(width) + size_t(x)) * 4,
                        slabs + hg_slab_index(s, uint32_t(slab_tiles)) * 4, 4 * sizeof(float));
        }
    return HG_OK;
}

}  // extern "C"
