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
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "halogen_abi.h"
#include "hg_ctx.h"
#include "hg_layout.h"

struct hg_comm {
    int32_t n_ranks = 0;
    int32_t transport = HG_COMM_RCCL;
    std::string err;
    struct Member {
        hg_ctx* ctx = nullptr;
        int32_t rank = 0;
        ncclComm_t nccl = nullptr;  // RCCL transport
        hipEvent_t done = nullptr;  // peer transport: this rank's slab copy is complete (root: slabs free to write)
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
#define HG_CNCCL(comm, call)                                                                                     \
    do {                                                                                                         \
        ncclResult_t r_ = (call);                                                                                \
        if (r_ != ncclSuccess) return cfail((comm), HG_E_COMM, "%s failed: %s", #call, ncclGetErrorString(r_)); \
    } while (0)

int64_t local_tiles(int64_t total, int32_t rank, int32_t n) {
    return total > rank ? (total - rank + n - 1) / n : 0;
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

// Every member context must be tiled as (its rank, n_ranks) and hold a target of the same size.
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

}  // namespace

// Row-major image from the root's own accumulator (tiles of the root rank) and the received slabs (other ranks):
// global tile g = (y/8)*tiles_x + x/8 lives on rank g % n at local slot g / n, pixel (x&7) + 8*(y&7) of it.
__global__ __launch_bounds__(256) void hg_assemble_image(float4* __restrict__ image, const float4* __restrict__ own,
                                                         const float4* __restrict__ slabs, int32_t W, int32_t H,
                                                         int32_t tiles_x, int32_t n, int32_t root,
                                                         uint32_t slab_tiles) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= uint32_t(W) * uint32_t(H)) return;
    const uint32_t x = i % uint32_t(W), y = i / uint32_t(W);
    const uint32_t g = (y >> 3) * uint32_t(tiles_x) + (x >> 3);
    const uint32_t r = g % uint32_t(n), l = g / uint32_t(n);
    const size_t lane = (x & 7u) + 8u * (y & 7u);
    image[i] = r == uint32_t(root) ? own[size_t(l) * 64 + lane] : slabs[(size_t(r) * slab_tiles + l) * 64 + lane];
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
    hg_comm::Member mb;
    mb.ctx = ctx;
    mb.rank = rank;
    ncclUniqueId u;
    std::memcpy(u.internal, id, HG_COMM_ID_BYTES);
    if (hipSetDevice(ctx->device) != hipSuccess) {
        delete m;
        return HG_E_HIP;
    }
    const ncclResult_t r = ncclCommInitRank(&mb.nccl, n_ranks, u, rank);
    if (r != ncclSuccess) {
        ctx->err = std::string("ncclCommInitRank failed: ") + ncclGetErrorString(r);
        delete m;
        return HG_E_COMM;
    }
    m->members.push_back(mb);
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
        if (!distinct) {
            if (hipSetDevice(mb.ctx->device) != hipSuccess ||
                hipEventCreateWithFlags(&mb.done, hipEventDisableTiming) != hipSuccess) {
                hg_comm_destroy(m);
                return HG_E_HIP;
            }
        }
    }
    *out = m;
    return HG_OK;
}

int hg_comm_gather(hg_comm* m, int32_t root) {
    if (!m) return HG_E_INVALID;
    if (root < 0 || root >= m->n_ranks) return cfail(m, HG_E_INVALID, "root %d out of range", root);
    const hg_ctx* c0 = m->members.front().ctx;
    const int32_t W = c0->W, H = c0->H;
    for (const auto& mb : m->members)
        if (int rc = check_member(m, mb, W, H)) return rc;
    const int32_t n = m->n_ranks;
    const int64_t total = int64_t(c0->tiles_x) * c0->tiles_y;
    const int64_t slab_tiles = local_tiles(total, 0, n);  // rank 0 holds the most tiles
    const size_t slab_floats = size_t(slab_tiles) * 64 * 4;
    hg_comm::Member* rootm = nullptr;
    for (auto& mb : m->members)
        if (mb.rank == root) rootm = &mb;
    if (rootm) {  // this process holds the root: staging slabs and the image on its device
        HG_CHIP(m, hipSetDevice(rootm->ctx->device));
        if (m->buf_device != rootm->ctx->device) {  // a root on another device: its own staging
            HG_CHIP(m, hipDeviceSynchronize());
            for (DevBuf* b : {&m->slabs, &m->image}) {
                if (b->p) (void)hipFree(b->p);
                *b = DevBuf{};
            }
            m->buf_device = rootm->ctx->device;
        }
        if (int rc = ensure_buf(m, m->slabs, size_t(n) * slab_floats * sizeof(float))) return rc;
        if (int rc = ensure_buf(m, m->image, size_t(W) * size_t(H) * sizeof(float4))) return rc;
    }
    m->root = -1;  // valid again once the assembly is enqueued
    if (m->transport == HG_COMM_RCCL) {
        HG_CNCCL(m, ncclGroupStart());
        for (auto& mb : m->members) {
            const size_t cnt = size_t(local_tiles(total, mb.rank, n)) * 64 * 4;
            if (mb.rank == root) {
                for (int32_t r = 0; r < n; ++r) {
                    const size_t rc = size_t(local_tiles(total, r, n)) * 64 * 4;
                    if (r == root || rc == 0) continue;
                    float* dst = static_cast<float*>(m->slabs.p) + size_t(r) * slab_floats;
                    HG_CNCCL(m, ncclRecv(dst, rc, ncclFloat32, r, mb.nccl, mb.ctx->stream));
                }
            } else if (cnt) {
                HG_CNCCL(m, ncclSend(mb.ctx->acc.p, cnt, ncclFloat32, root, mb.nccl, mb.ctx->stream));
            }
        }
        HG_CNCCL(m, ncclGroupEnd());
    } else {  // peer transport: every member is in this process and rootm is set
        // the slabs are free once the root's previous assembly has read them
        HG_CHIP(m, hipEventRecord(rootm->done, rootm->ctx->stream));
        for (auto& mb : m->members) {
            if (mb.rank == root) continue;
            HG_CHIP(m, hipSetDevice(mb.ctx->device));
            HG_CHIP(m, hipStreamWaitEvent(mb.ctx->stream, rootm->done, 0));
            const size_t bytes = size_t(local_tiles(total, mb.rank, n)) * 64 * sizeof(float4);
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

int hg_comm_readback(hg_comm* m, float* rgba, size_t n_floats) {
    if (!m || !rgba) return HG_E_INVALID;
    if (m->root < 0 || !m->root_ctx) return cfail(m, HG_E_INVALID, "no gathered image in this process");
    if (n_floats < size_t(m->W) * size_t(m->H) * 4) return cfail(m, HG_E_INVALID, "readback buffer too small");
    hg_ctx* rc = m->root_ctx;
    HG_CHIP(m, hipSetDevice(rc->device));
    HG_CHIP(m, hipMemcpyAsync(rgba, m->image.p, size_t(m->W) * size_t(m->H) * sizeof(float4), hipMemcpyDeviceToHost,
                              rc->stream));
    HG_CHIP(m, hipStreamSynchronize(rc->stream));
    return HG_OK;
}

int hg_comm_transport(const hg_comm* m) { return m ? m->transport : HG_E_INVALID; }

const char* hg_comm_last_error(const hg_comm* m) { return m ? m->err.c_str() : "null communicator"; }

void hg_comm_destroy(hg_comm* m) {
    if (!m) return;
    for (auto& mb : m->members) {
        if (mb.ctx) {
            (void)hipSetDevice(mb.ctx->device);
            (void)hipStreamSynchronize(mb.ctx->stream);
        }
        if (mb.nccl) (void)ncclCommDestroy(mb.nccl);
        if (mb.done) (void)hipEventDestroy(mb.done);
    }
    if (m->root_ctx) (void)hipSetDevice(m->root_ctx->device);
    if (m->slabs.p) (void)hipFree(m->slabs.p);
    if (m->image.p) (void)hipFree(m->image.p);
    delete m;
}

}  // extern "C"
