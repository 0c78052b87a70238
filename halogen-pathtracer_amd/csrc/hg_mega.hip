// hg_mega.hip — the megakernels of the hot path: the streaming kernel (default for deep BLAS), the regenerating
// kernel (default otherwise) and the lockstep kernel (HG_KERNEL_MEGA: debug views, large-maxBounces fallback).
//
// Reference: Assets/Scripts/Halogen Shaders/HalgoenCompute.compute, kernel HalogenCompute (:1015-1063) with
// the accumulation blit (AccumulationShader.shader:27-34) fused as its epilogue.  One wave64 = one 8x8 pixel
// tile; the BLAS stack lives in LDS ([depth][lane]).  The lockstep kernel below is the simplest faithful form:
// each lane runs all n_frames frames of its pixel back to back.
#include <hip/hip_runtime.h>

#include "hg_device.h"

using namespace hgd;

// kDebug: the debug views (HalogenDebugMode 1-5) get their own instantiation so the production kernel's register
// allocation does not pay for trace_ray_debug.
template <bool kCounters, bool kDebug>
__global__ __launch_bounds__(256, HG_LOCK_WAVES) void hg_trace_kernel(const HgKernelParams kp) {
    const uint32_t lane = threadIdx.x & 63u;
    const int local_tile = int(xcd_block(blockIdx.x, gridDim.x)) * int(blockDim.x >> 6) + int(threadIdx.x >> 6);
    const int gtile = kp.rank + local_tile * kp.n_ranks;
    const uint32_t px = uint32_t(gtile % kp.tiles_x) * HG_TILE + (lane & 7u);
    const uint32_t py = uint32_t(gtile / kp.tiles_x) * HG_TILE + (lane >> 3);
    const bool active = local_tile < kp.n_local_tiles && px < kp.Wu && py < kp.Hu;
    Counters c{0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t paths = 0;
    if (active) {
        const MegaStack stk{threadIdx.x, blockDim.x, kp.spill + blockIdx.x * blockDim.x + threadIdx.x,
                            kp.spill_stride};
        const size_t slot = size_t(local_tile) * 64 + lane;
        // HalogenCompute :1023-1033
        const float ndcx = (float(px) / kp.W) * 2.0f - 1.0f;
        const float ndcy = (float(py) / kp.H) * 2.0f - 1.0f;
        const uint32_t pixel_id = pcg_hash(px + py * kp.Wu);
        for (int f = 0; f < kp.n_frames; ++f) {
            const int32_t fc = kp.accumulate ? kp.first_frame + f : 1;
            Sampler smp{uint32_t(fc), pixel_id, 0u};
            MediumStack ms{0ull, 0};
            f3 color = mk(0, 0, 0);
            for (uint32_t s = 0; s < kp.spp; ++s) {
                const Ray r = camera_ray(kp, smp, ndcx, ndcy);
                paths++;
                if (!kDebug) color = color + trace_ray(kp, smp, ms, r, c, stk);
                else color = color + trace_ray_debug(kp, smp, ms, r, c, stk);
            }
            const float sppf = float(kp.spp);
            color = mk(color.x / sppf, color.y / sppf, color.z / sppf);
            float4 acc = kp.acc[slot];  // read-modify-write per frame: 32 B, keeps 4 VGPRs free while tracing
            if (kp.accumulate) {  // AccumulationShader.shader:33, w = 1/FrameCount
                const float w = rcp_exact(float(fc));
                const float k = 1.0f - w;
                acc.x = acc.x * k + color.x * w;
                acc.y = acc.y * k + color.y * w;
                acc.z = acc.z * k + color.z * w;
                acc.w = acc.w * k + 1.0f * w;
            } else {
                acc = make_float4(color.x, color.y, color.z, 1.0f);
            }
            kp.acc[slot] = acc;
        }
    }
    if (kCounters) {
        // every ray transforms into every mesh and prefilters every sphere: those counts follow from c.rays
        const uint32_t v[9] = {paths, c.rays, c.tri, c.aabb, c.rays * uint32_t(kp.n_meshes),
                               c.rays * uint32_t(kp.n_spheres), c.hits, c.node_rounds, c.tri_rounds};
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint32_t s = wave_sum(v[k]);
            if (lane == 0 && s) atomicAdd(kp.counters + k, (unsigned long long)s);
        }
        const uint32_t pm = wave_sum(c.primary_miss);
        if (lane == 0 && pm) atomicAdd(kp.counters + 16, (unsigned long long)pm);
    }
}

size_t hg_mega_lds_bytes(uint32_t stack_depth, int block) {
    return size_t(stack_depth < HG_MEGA_LDS_STACK ? stack_depth : HG_MEGA_LDS_STACK) * size_t(block) *
           sizeof(uint32_t);
}

// Regenerating variant (HG_KERNEL_MEGA_REGEN): each loop iteration runs ONE bounce (get_ray_intersection + one
// body of trace_ray's loop, :887-945) for every lane; a lane whose path ended starts its next sample / frame right
// away (blending a finished frame into the accumulator), so lanes never idle until the longest path of their wave
// ends — at the price of desynchronised bounce depths (less coherent node fetches).  Path state is packed to keep
// the traversal's register budget: bounceTypes[3] + the bounce index in one word (host guarantees maxBounces <=
// HG_REGEN_MAX_BOUNCES), frame + sample index in another (n_frames, spp < 2^16, host-chunked), the pixel's ndc /
// accumulator slot recomputed at each regeneration.
// Per-lane path state parked in LDS (RowVec3 / RowVec4 rows, hg_device.h): the throughput, radiance and sample sum
// are touched once per bounce, so they stay out of the registers the traversal needs.
constexpr uint32_t kRegenLdsState = 9;  // words per lane: throughput, radiance, sample sum
// Streaming kernel: one more word per lane (row 9, unused since the round-2 LDS accumulator was retired: the leaf-share
// rows stay 64-bit aligned at row 10).
constexpr uint32_t kStreamLdsState = 10;
// Streaming kernel LDS rows (one wave per workgroup, RowVec / RowStack): throughput 0-2, path colour 3-5, sample sum
// 6-8, the distributed leaf test 10-12, the traversal stack from row 13.
constexpr uint32_t kRowThr = 0, kRowCol = 3, kRowSum = 6, kRowLeaf = kStreamLdsState;
[[maybe_unused]] constexpr uint32_t kRowSort = 9;  // HG_RAY_SORT builds: the lane-permutation scratch row
constexpr uint32_t kRowCache = kRowLeaf + 3, kRowStack = kRowCache + HG_NODE_CACHE / 4;  // node cache rows, stack
static_assert(kRowCache == HG_STREAM_CACHE_ROW && HG_NODE_CACHE % 4 == 0, "stream LDS rows");
constexpr uint32_t kRegenRowStack = kRegenLdsState;  // regenerating kernel: rows 0-8 as above, the stack from row 9

// Cost-ordered dispatch (HgKernelParams::tile_order): the wave's tile, read through the scalar cache (the order is
// written by hg_order_tiles before this launch and never during it).
__device__ __forceinline__ int ordered_tile(const HgKernelParams& kp, uint32_t w) {
    if (!kp.tile_order) return int(w);
#if HG_TILE_ORDER_SCALAR
    typedef const __attribute__((address_space(4))) uint32_t* cu32p;
    return int(((cu32p)(uintptr_t)kp.tile_order)[__builtin_amdgcn_readfirstlane(w)]);
#else
    return int(kp.tile_order[w]);
#endif
}
// The wave's work unit (tile, frame chunk).  Tile-index order: chunk-major (wave w: tile w mod tiles, chunk
// w / tiles).  Cost order with HG_UNIT_TILE_MAJOR: tile-major (wave w: tile order[w / split], chunk w mod split), so
// a tile's chunks run side by side and the most expensive tiles' chunks all start first.  Waves past the last unit
// get chunk = split (no work).
__device__ __forceinline__ void wave_unit(const HgKernelParams& kp, uint32_t gw, uint32_t nlt, uint32_t split,
                                          int& tile, uint32_t& chunk) {
#if HG_UNIT_TILE_MAJOR
    if (kp.tile_order) {
        const uint32_t w = gw / split;
        tile = w < nlt ? ordered_tile(kp, w) : 0;
        chunk = w < nlt ? gw % split : split;
        return;
    }
#endif
    tile = ordered_tile(kp, gw % nlt);
    chunk = gw / nlt;
}

// The wave's clock time (s_memtime cycles), added to its tile's 64-bit cost for the next launch's order (no wrap for
// any launch: 2^64 cycles).  The start time and the tile wait in LDS, not in registers that would stay live across
// the whole kernel.
__shared__ uint64_t hg_wave_t0[4];
__shared__ unsigned long long* hg_wave_cost[4];  // &tile_cost[tile], null: not recorded
__device__ __forceinline__ void tile_cost_begin(const HgKernelParams& kp, uint32_t lane, int tile, bool valid) {
    if (lane == 0) {
        hg_wave_cost[threadIdx.x >> 6] = kp.tile_cost && valid ? kp.tile_cost + tile : nullptr;
        hg_wave_t0[threadIdx.x >> 6] = wave_clock();
    }
}
// a global-memory atomic add through a pointer kept in LDS (a generic pointer would compile to a FLAT atomic)
__device__ __forceinline__ void cost_add(unsigned long long* p, uint64_t v) {
    typedef __attribute__((address_space(1))) unsigned long long* gptr;
    __hip_atomic_fetch_add((gptr)(uintptr_t)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void record_tile_cost(uint32_t lane) {
    if (lane != 0) return;
    unsigned long long* const p = hg_wave_cost[threadIdx.x >> 6];
    if (p) cost_add(p, wave_clock() - hg_wave_t0[threadIdx.x >> 6]);
}

// RayColor / SamplesPerPixel (:1060); x / 1 == x exactly (NaN and signed zeros included), so spp 1 skips the divisions
__device__ __forceinline__ f3 sample_mean(const HgKernelParams& kp, f3 sum) {
    if (kp.spp == 1) return sum;
    const float sppf = float(kp.spp);
    return mk(sum.x / sppf, sum.y / sppf, sum.z / sppf);
}

// (pixel, frame) items of a wave's tile (HG_STREAM_ITEMS / HG_REGEN_ITEMS): with the v pixels of the tile inside the
// image (a w x h rectangle; all 64 for a whole tile), item k is valid pixel k mod v of frame f_begin + k / v.  Lane l
// starts with item l; a lane whose frame is done takes the next unassigned item (its rank among the wave's lanes that
// need one), so the lanes stay busy until the tile's items run out instead of each waiting for its own pixel's
// slowest frames.  Every frame's colour goes to frame_color and hg_blend_frames applies the accumulation blend in
// frame order afterwards: the same operations in the same order as a lane tracing its pixel's frames in turn.
__shared__ uint32_t hg_next_item;  // items of the wave's tile handed out so far (one wave per workgroup)
struct TileItems {
    uint32_t tx0, ty0, tw, nv, n_items, f_begin;  // wave-uniform (scalar registers)
#if HG_ITEMS_PIXEL_MAJOR
    uint32_t nf;  // frames of the chunk
#endif
    __device__ TileItems() : tx0(0), ty0(0), tw(0), nv(0), n_items(0), f_begin(0) {  // unused (kQueue kernels)
#if HG_ITEMS_PIXEL_MAJOR
        nf = 1u;
#endif
    }
    __device__ TileItems(const HgKernelParams& kp, int local_tile, bool valid, uint32_t fb, uint32_t fe, uint32_t lane) {
        const int g = __builtin_amdgcn_readfirstlane(kp.rank + local_tile * kp.n_ranks);
        tx0 = uint32_t(g % kp.tiles_x) * HG_TILE;
        ty0 = uint32_t(g / kp.tiles_x) * HG_TILE;
        tw = __builtin_amdgcn_readfirstlane(min(uint32_t(HG_TILE), kp.Wu - min(kp.Wu, tx0)));
        const uint32_t th = __builtin_amdgcn_readfirstlane(min(uint32_t(HG_TILE), kp.Hu - min(kp.Hu, ty0)));
        nv = tw * th;
        n_items = __builtin_amdgcn_readfirstlane(valid && fe > fb ? nv * (fe - fb) : 0u);
        f_begin = fb;
#if HG_ITEMS_PIXEL_MAJOR
        nf = __builtin_amdgcn_readfirstlane(fe > fb ? fe - fb : 1u);
#endif
        if (lane == 0) hg_next_item = 64u;  // lane l starts with item l
        wave_lds_sync();
    }
    // item k -> its pixel within the tile (x + 8 y) and its frame: shifts for a whole tile, divisions at the edge
    __device__ __forceinline__ void get(uint32_t k, uint32_t& pix, uint32_t& frame) const {
        uint32_t q;
#if HG_ITEMS_PIXEL_MAJOR  // item k -> valid pixel k / nf, frame k mod nf (a wave's lanes on one pixel's frames)
        uint32_t i;
        if ((nf & (nf - 1u)) == 0u) {
            const uint32_t lg = uint32_t(__builtin_ctz(nf));
            i = k >> lg;
            q = k & (nf - 1u);
        } else {
            i = k / nf;
            q = k - i * nf;
        }
        pix = nv == 64u ? i : (i % tw) + 8u * (i / tw);
        frame = f_begin + q;
        return;
#endif
        if (nv == 64u) {
            pix = k & 63u;
            q = k >> 6;
        } else {
            q = k / nv;
            const uint32_t i = k - q * nv;
            pix = (i % tw) + 8u * (i / tw);
        }
        frame = f_begin + q;
    }
    // Called by exactly the lanes that need an item (the active lanes): they take the next items in lane order.  The
    // first of them advances the LDS counter with one atomic add and its old value goes to the others by
    // readfirstlane.  Returns the item's index k, k >= n_items when the tile's items are all handed out; the caller
    // decodes k with get() inside its branch (decoded here, the frame was held across a control-flow merge and spilled
    // to scratch at every take).
    __device__ __forceinline__ uint32_t take_here() const {
        const uint64_t m = __builtin_amdgcn_read_exec();
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
        uint32_t base = 0;
        if (rank == 0u) base = atomicAdd(&hg_next_item, uint32_t(__builtin_popcountll(m)));
        base = __builtin_amdgcn_readfirstlane(base);
        return base + rank;
    }
};

// LDS words read / written by different lanes of the wave (see the queue's note below)
__device__ __forceinline__ uint32_t lds_get(uint32_t& x) {
    return __hip_atomic_load(&x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_put(uint32_t& x, uint32_t v) {
    __hip_atomic_store(&x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// (pixel, frame) items of a streaming wave's units (launches without the queue).  The wave traces the nu units
// [u0, u0 + nu) of the launch's unit order (wave_unit; nu = kp.wave_units <= HG_WAVE_UNITS_LIMIT, more than one only
// without a frame split, where unit u is tile ordered_tile(u) with all the launch's frames), their items numbered one
// unit after another and pixel-major within a unit as in TileItems.  A lane that finishes a frame takes the wave's
// next item whichever unit holds it, so the wave's lanes drain once per nu tiles instead of once per tile; which wave
// traces an item changes nothing (every item runs with its own pixel's and frame's inputs and writes its own colour
// slot).  A lane's item is held as v = unit j << 6 | pixel (x + 8 y); the units' tiles and image origins sit in the
// wave's LDS (the kernel's scalar registers are all taken), read once when a path starts and once when it ends.
__shared__ uint32_t hg_unit_tile[HG_WAVE_UNITS_LIMIT];  // unit j's local tile
__shared__ uint32_t hg_unit_org[HG_WAVE_UNITS_LIMIT];   // its image origin x | y << 16
__shared__ uint32_t hg_unit_shape;                      // unit 0's valid width | valid pixels << 8
struct UnitItems {
    uint32_t nu, nf, f_begin, n_items, full;  // wave-uniform (scalar registers)
    __device__ UnitItems() : nu(0), nf(1), f_begin(0), n_items(0), full(1) {}  // unused (kQueue)
    __device__ UnitItems(const HgKernelParams& kp, uint32_t u_first, int first_tile, bool valid, uint32_t fb,
                         uint32_t fe, uint32_t lane) {
        const uint32_t nlt = uint32_t(kp.n_local_tiles), u0 = __builtin_amdgcn_readfirstlane(u_first);
        nu = valid ? (kp.wave_units > 1u && u0 < nlt ? min(min(kp.wave_units, uint32_t(HG_WAVE_UNITS_LIMIT)), nlt - u0)
                                                     : 1u)
                   : 0u;
        nu = __builtin_amdgcn_readfirstlane(nu);
        nf = __builtin_amdgcn_readfirstlane(fe > fb ? fe - fb : 1u);
        f_begin = fb;
        n_items = 0u;
        full = 1u;
        for (uint32_t j = 0; j < nu; ++j) {
            const uint32_t t = __builtin_amdgcn_readfirstlane(j == 0u ? first_tile : ordered_tile(kp, u0 + j));
            uint32_t tx0, ty0, tw, th;
            tile_rect(kp, t, tx0, ty0, tw, th);
            if (lane == 0) {
                hg_unit_tile[j] = t;
                hg_unit_org[j] = tx0 | (ty0 << 16);
                if (j == 0u) hg_unit_shape = tw | ((tw * th) << 8);
            }
            n_items += tw * th * (fe > fb ? fe - fb : 0u);
            full &= tw * th == 64u ? 1u : 0u;
        }
        n_items = __builtin_amdgcn_readfirstlane(n_items);
        full = __builtin_amdgcn_readfirstlane(full);
        if (lane == 0) hg_next_item = 64u;  // lane l starts with item l
        wave_lds_sync();
    }
    __device__ static __forceinline__ void tile_rect(const HgKernelParams& kp, uint32_t t, uint32_t& tx0, uint32_t& ty0,
                                                     uint32_t& tw, uint32_t& th) {
        const uint32_t g = uint32_t(kp.rank) + t * uint32_t(kp.n_ranks);
        const uint32_t ty = g / uint32_t(kp.tiles_x);
        tx0 = (g - ty * uint32_t(kp.tiles_x)) * HG_TILE;
        ty0 = ty * HG_TILE;
        tw = min(uint32_t(HG_TILE), kp.Wu - min(kp.Wu, tx0));
        th = min(uint32_t(HG_TILE), kp.Hu - min(kp.Hu, ty0));
    }
    // item k -> v (unit j << 6 | pixel) and its frame
    __device__ __forceinline__ void get(const HgKernelParams& kp, uint32_t k, uint32_t& v, uint32_t& frame) const {
        uint32_t j = 0u, kk = k, nv = 64u, tw = 8u;
        if (full) {
            if ((nf & (nf - 1u)) == 0u) {
                const uint32_t lg = 6u + uint32_t(__builtin_ctz(nf));
                j = k >> lg;
                kk = k & ((1u << lg) - 1u);
            } else {
                j = k / (64u * nf);
                kk = k - j * (64u * nf);
            }
        } else {  // a tile at the image edge (only ever a wave's one unit: the runtime gives such images one tile per wave)
            const uint32_t sh = lds_get(hg_unit_shape);
            tw = sh & 0xFFu;
            nv = sh >> 8;
        }
        uint32_t i, f;
        if ((nf & (nf - 1u)) == 0u) {
            const uint32_t lg = uint32_t(__builtin_ctz(nf));
            i = kk >> lg;
            f = kk & (nf - 1u);
        } else {
            i = kk / nf;
            f = kk - i * nf;
        }
        v = (j << 6) | (nv == 64u ? i : (i % tw) + 8u * (i / tw));
        frame = f_begin + f;
    }
    __device__ __forceinline__ uint32_t slot(uint32_t v) const {
        return nu <= 1u ? (lds_get(hg_unit_tile[0]) * 64u + v) : lds_get(hg_unit_tile[v >> 6]) * 64u + (v & 63u);
    }
    __device__ __forceinline__ void pixel(uint32_t v, uint32_t& x, uint32_t& y) const {
        const uint32_t o = lds_get(hg_unit_org[v >> 6]);
        x = (o & 0xFFFFu) + (v & 7u);
        y = (o >> 16) + ((v >> 3) & 7u);
    }
    __device__ __forceinline__ uint32_t take_here() const {
        const uint64_t m = __builtin_amdgcn_read_exec();
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
        uint32_t base = 0;
        if (rank == 0u) base = atomicAdd(&hg_next_item, uint32_t(__builtin_popcountll(m)));
        base = __builtin_amdgcn_readfirstlane(base);
        return base + rank;
    }
    // the wave's clock since tile_cost_begin, shared out over its units' tiles (the first one's pointer is in LDS)
    __device__ __forceinline__ void record_cost(const HgKernelParams& kp, uint32_t lane) const {
        if (nu <= 1u) {
            record_tile_cost(lane);
            return;
        }
        if (lane != 0 || !hg_wave_cost[threadIdx.x >> 6]) return;
        const uint64_t share = (wave_clock() - hg_wave_t0[threadIdx.x >> 6]) / nu;
        for (uint32_t j = 0; j < nu; ++j) cost_add(kp.tile_cost + lds_get(hg_unit_tile[j]), share);
    }
};

// Cost order (hg_render, per trace stream): tile_order = the local tiles, most expensive first, then the costs are
// cleared for the next launches.  A counting sort over 1024 log-scale cost buckets (16 per octave of the wave-clock
// cost: bucket 0 the most expensive; two tiles share one only within ~4 % of each other), in two launches of one-wave
// workgroups (1,024 tiles each) with 8-12 KB of LDS and few registers, so that they fit on CUs beside the persistent
// trace waves of the other streams (round 3's single 1,024-thread, 36-KB workgroup waited for a whole CU to drain:
// ~1 ms per sort at the one-dispatch-per-frame operating point):
//   hg_order_hist     each workgroup histograms its tiles in LDS and adds the counts to the global histogram;
//   hg_order_scatter  each workgroup derives the buckets' starts (exclusive prefix of the global histogram), claims its
//                     share of every bucket with one global atomic per (workgroup, bucket) and places its tiles there;
//                     the last workgroup to finish clears the histogram and the claims for the next sort.
// Within a bucket the order is not tile-index order (it depends on which workgroup claims first): no result depends on
// the order (tiles are independent), only the drain tail.  The order is a permutation of the tiles whenever the costs
// hold still during the sort (the runtime sorts a stream's own costs on that stream); HG_CHECK_EXEC builds also verify
// that (hg_order_verify) and count every placement out of range into hg_counters.order_faults.
struct HgOrderScratch {  // per trace stream, zeroed at allocation; every sort leaves it zeroed again
    uint32_t hist[1024];   // tiles per bucket
    uint32_t claim[1024];  // tiles per bucket claimed by workgroups so far
    uint32_t done;         // workgroups of the scatter launch finished
    uint32_t pad[31];
};
static_assert(sizeof(HgOrderScratch) == 8320, "order scratch");
constexpr uint32_t kOrderTilesPerGroup = 1024;

__device__ __forceinline__ uint32_t order_bucket(unsigned long long c) {
    if (c < 2ull) return 1023u;
    const uint32_t e = 63u - uint32_t(__builtin_clzll(c));                          // 1..63
    const uint32_t m = uint32_t(e >= 4u ? (c >> (e - 4u)) : (c << (4u - e))) & 15u;  // the 4 bits after the leading 1
    return 1023u - (e * 16u + m);
}

__global__ __launch_bounds__(64) void hg_order_hist(const unsigned long long* __restrict__ cost, uint32_t n,
                                                    HgOrderScratch* __restrict__ sc) {
    __shared__ uint32_t h[1024];
    const uint32_t t = threadIdx.x, base = blockIdx.x * kOrderTilesPerGroup;
    for (uint32_t b = t; b < 1024u; b += 64u) h[b] = 0u;
    __syncthreads();
    for (uint32_t k = t; k < kOrderTilesPerGroup && base + k < n; k += 64u) atomicAdd(&h[order_bucket(cost[base + k])], 1u);
    __syncthreads();
    for (uint32_t b = t; b < 1024u; b += 64u)
        if (h[b]) atomicAdd(&sc->hist[b], h[b]);
}

__global__ __launch_bounds__(64) void hg_order_scatter(unsigned long long* __restrict__ cost, uint32_t* __restrict__ order,
                                                       uint32_t n, HgOrderScratch* __restrict__ sc,
                                                       unsigned long long* __restrict__ faults) {
    __shared__ uint32_t pos[1024];  // bucket -> next place of this workgroup's tiles
    __shared__ uint32_t cnt[1024];  // bucket -> this workgroup's tiles
    const uint32_t t = threadIdx.x, base = blockIdx.x * kOrderTilesPerGroup;
    // exclusive prefix of the global histogram: lane t sums buckets [16t, 16t + 16), a wave scan of the 64 sums
    uint32_t run = 0;
    for (uint32_t j = 0; j < 16u; ++j) {
        const uint32_t v = __hip_atomic_load(&sc->hist[16u * t + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pos[16u * t + j] = run;
        run += v;
    }
    uint32_t incl = run;
    for (uint32_t d = 1; d < 64u; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d);
        if (t >= d) incl += o;
    }
    const uint32_t excl = incl - run;
    for (uint32_t j = 0; j < 16u; ++j) {
        pos[16u * t + j] += excl;
        cnt[16u * t + j] = 0u;
    }
    __syncthreads();
    for (uint32_t k = t; k < kOrderTilesPerGroup && base + k < n; k += 64u) atomicAdd(&cnt[order_bucket(cost[base + k])], 1u);
    __syncthreads();
    for (uint32_t b = t; b < 1024u; b += 64u)  // this workgroup's share of bucket b
        if (cnt[b]) pos[b] += atomicAdd(&sc->claim[b], cnt[b]);
    __syncthreads();
    uint32_t bad = 0;
    for (uint32_t k = t; k < kOrderTilesPerGroup && base + k < n; k += 64u) {
        const uint32_t i = base + k;
        const uint32_t p = atomicAdd(&pos[order_bucket(cost[i])], 1u);
        if (p < n) order[p] = i;  // always, while the costs hold still during the sort
        else ++bad;
        cost[i] = 0ull;
    }
#if HG_CHECK_EXEC
    if (bad && faults) atomicAdd(faults, (unsigned long long)bad);
#else
    (void)bad;
    (void)faults;
#endif
    __syncthreads();
    // the last workgroup out clears the histogram and the claims (every other one has read them: release / acquire)
    uint32_t last = 0;
    if (t == 0)
        last = __hip_atomic_fetch_add(&sc->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u;
    last = __builtin_amdgcn_readfirstlane(last);
    if (last) {
        for (uint32_t b = t; b < 1024u; b += 64u) {
            __hip_atomic_store(&sc->hist[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&sc->claim[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (t == 0) __hip_atomic_store(&sc->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

#if HG_CHECK_EXEC
// HG_CHECK_EXEC builds: the order must be a permutation of [0, n).  seen[] (n words, zero) counts each tile's places;
// the second kernel counts tiles placed other than once into *faults and zeroes seen[] again.
__global__ __launch_bounds__(64) void hg_order_verify_mark(const uint32_t* __restrict__ order, uint32_t n,
                                                           uint32_t* __restrict__ seen,
                                                           unsigned long long* __restrict__ faults) {
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = order[i];
    if (v < n) atomicAdd(&seen[v], 1u);
    else atomicAdd(faults, 1ull);
}
__global__ __launch_bounds__(64) void hg_order_verify_count(uint32_t n, uint32_t* __restrict__ seen,
                                                            unsigned long long* __restrict__ faults) {
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= n) return;
    if (seen[i] != 1u) atomicAdd(faults, 1ull);
    seen[i] = 0u;
}
#endif

size_t hg_order_scratch_bytes(uint32_t n) {
    return sizeof(HgOrderScratch) + (HG_CHECK_EXEC ? size_t(n) * sizeof(uint32_t) : 0);
}

// scratch: hg_order_scratch_bytes(n) bytes, zeroed when allocated; faults: hg_counters.order_faults (check builds)
hipError_t hg_launch_order_tiles(unsigned long long* cost, uint32_t* order, uint32_t n, void* scratch,
                                 unsigned long long* faults, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    HgOrderScratch* sc = static_cast<HgOrderScratch*>(scratch);
    const dim3 g{(n + kOrderTilesPerGroup - 1) / kOrderTilesPerGroup};
    hipLaunchKernelGGL(hg_order_hist, g, dim3(64), 0, stream, cost, n, sc);
    hipLaunchKernelGGL(hg_order_scatter, g, dim3(64), 0, stream, cost, order, n, sc, faults);
#if HG_CHECK_EXEC
    uint32_t* seen = reinterpret_cast<uint32_t*>(sc + 1);
    hipLaunchKernelGGL(hg_order_verify_mark, dim3((n + 63) / 64), dim3(64), 0, stream, order, n, seen, faults);
    hipLaunchKernelGGL(hg_order_verify_count, dim3((n + 63) / 64), dim3(64), 0, stream, n, seen, faults);
#endif
    return hipGetLastError();
}

template <bool kCounters, bool kMeshLds>
__global__ __launch_bounds__(HG_STREAM_LB, HG_MEGA_WAVES) void hg_trace_regen_kernel(const HgKernelParams kp) {
    const uint32_t lane = threadIdx.x & 63u;
    if (kMeshLds) {  // the wave's copy of the mesh records (mesh_f4, hg_device.h)
        mesh_lds_fill(kp, lane);
        wave_lds_sync();
    }
    // wave -> (tile, frame chunk): with frame_split == 1 the wave index is the tile
    // one wave per workgroup (launched with 64 threads): wave = workgroup; LDS rows as the streaming kernel's
    const uint32_t gw = xcd_block(blockIdx.x, gridDim.x);
    const uint32_t nlt = uint32_t(kp.n_local_tiles), split = uint32_t(kp.frame_split);
    int local_tile;
    uint32_t chunk;
    wave_unit(kp, gw, nlt, split, local_tile, chunk);
    tile_cost_begin(kp, lane, local_tile, chunk < split);
    const uint32_t f_begin = uint32_t((uint64_t(chunk) * uint32_t(kp.n_frames)) / split);
    const uint32_t f_end = uint32_t((uint64_t(chunk + 1) * uint32_t(kp.n_frames)) / split);
    const RowStack<HG_MEGA_LDS_STACK, kRegenRowStack> stk{lane, kp.spill + blockIdx.x * 64u + lane, kp.spill_stride};
    const RowVec3<kRowThr> s_thr{lane};
    const RowVec3<kRowCol> s_col{lane};
    const RowVec3<kRowSum> s_sum{lane};
    bool work;
    uint32_t px, py;
    {
        const int gtile = kp.rank + local_tile * kp.n_ranks;
        px = uint32_t(gtile % kp.tiles_x) * HG_TILE + (lane & 7u);
        py = uint32_t(gtile / kp.tiles_x) * HG_TILE + (lane >> 3);
        work = chunk < split && px < kp.Wu && py < kp.Hu && f_end > f_begin;
    }
    Counters c{0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t paths = 0;
    uint32_t fs = f_begin << 16;  // frame index << 16 | sample index
    uint32_t bounce = 0;          // diffuse | glossy << 8 | transmission << 16 | bounce index << 24
    Sampler smp{kp.accumulate ? uint32_t(kp.first_frame) + f_begin : 1u, pcg_hash(px + py * kp.Wu), 0u};
    MediumStack ms{0ull, 0};
    Ray ray{mk(0, 0, 0), mk(0, 0, 1)};
    float acc_rough = 0.0f;
#if HG_REGEN_ITEMS
    const TileItems items(kp, local_tile, chunk < split, f_begin, f_end, lane);
    uint32_t pix = lane;  // the item's pixel within the tile (x + 8 y)
    if (lane < items.n_items) {  // item `lane`
        uint32_t f;
        items.get(lane, pix, f);
        px = items.tx0 + (pix & 7u);
        py = items.ty0 + (pix >> 3);
        fs = f << 16;
        smp = Sampler{kp.accumulate ? uint32_t(kp.first_frame) + f : 1u, pcg_hash(px + py * kp.Wu), 0u};
    }
    work = lane < items.n_items;
#else
    const uint32_t pix = lane;
#endif
    if (work) {
        ray = camera_ray(kp, smp, (float(px) / kp.W) * 2.0f - 1.0f, (float(py) / kp.H) * 2.0f - 1.0f);  // :1023-1033
        paths++;
        s_thr.set(mk(1, 1, 1));
        s_col.set(mk(0, 0, 0));
        s_sum.set(mk(0, 0, 0));
    }
    uint64_t cyc_trav = 0, cyc_shade = 0;  // wave clock (s_memtime) per phase, counting instantiation only
    while (__any(work)) {
        const uint64_t t0 = kCounters ? wave_clock() : 0;
        const bool was_work = work;
        uint64_t t1 = 0;
        if (work) {
#if HG_REGEN_PRIO
            __builtin_amdgcn_s_setprio(1);
#endif
            const Hit hit = intersect<kMeshLds>(kp, ray, c, stk);
#if HG_REGEN_PRIO
            __builtin_amdgcn_s_setprio(0);
#endif
            if (kCounters) t1 = wave_clock();
            c.shade_rounds += wave_once();
            bool alive = false;
            f3 thr = s_thr.get(), col = s_col.get();
            if (hit.t < kp.far_) {  // :898-936
                c.hits++;
                const Mat mt = load_mat(kp, hit.mat);
                col = col + xyz(mt.emis_rough) * thr;
                uint32_t bt = 0;
                const f3 att = evaluate_hit(kp, smp, ms, ray, hit, mt, bt);
                bounce += 1u << (8u * bt);
                thr = thr * att;
                acc_rough += mt.emis_rough.w * thr.x;
                const float rr = smp.get1(ID_RR);
                smp.offset += BOUNCE_INC;
                const float contribution = fmaxf(fmaxf(thr.x, thr.y), thr.z);
                if (!(rr > contribution)) {
                    thr = thr * rcp_exact(contribution);
                    bounce += 1u << 24;
                    alive = (bounce >> 24) <= kp.max_bounces && !((bounce & 0xFFu) > kp.max_diff ||
                                                                 ((bounce >> 8) & 0xFFu) > kp.max_glossy ||
                                                                 ((bounce >> 16) & 0xFFu) > kp.max_trans);
                }
            } else {  // :941
                c.primary_miss += bounce == 0u;  // the path's camera ray (no bounce recorded yet)
                col = col + sample_sky(kp, ray.d, sky_level(kp, acc_rough)) * thr;
            }
            if (!alive) {
                // RayColor += trace_ray(...); spp 1: 0 + col == col (col starts at +0 and only has terms added: never -0)
                const bool one_sample = kp.spp == 1;
                f3 sum = one_sample ? col : s_sum.get() + col;
                ++fs;
                bool next = (fs & 0xFFFFu) < kp.spp;  // next sample: statics persist (:188-189)
                if (!next) {
                    const f3 color = sample_mean(kp, sum);
                    const size_t slot_i = size_t(uint32_t(local_tile)) * 64u + pix;
                    // this frame's colour, blended later in frame order: every launch of the trace pipeline (the runtime
                    // passes a colour buffer exactly then, and blends after every chunk of it, a 1-frame chunk included)
                    if (HG_REGEN_ITEMS || kp.frame_color != nullptr) {
                        fc_store(kp.frame_color + fc_index(kp, fs >> 16, slot_i),
                                 make_float4(color.x, color.y, color.z, 1.0f));
                    } else {
                        float4* slot = kp.acc + slot_i;
                        float4 acc = *slot;
                        if (kp.accumulate) {  // AccumulationShader.shader:33, w = 1/FrameCount
                            const float w = rcp_exact(float(smp.frame));
                            const float k = 1.0f - w;
                            acc = make_float4(acc.x * k + color.x * w, acc.y * k + color.y * w,
                                              acc.z * k + color.z * w, acc.w * k + 1.0f * w);
                        } else {
                            acc = make_float4(color.x, color.y, color.z, 1.0f);
                        }
                        *slot = acc;
                    }
                    fs = (fs & 0xFFFF0000u) + 0x10000u;
#if HG_REGEN_ITEMS
                    const uint32_t k = items.take_here();
                    if (k < items.n_items) {  // the next (pixel, frame) item: statics reset as for a dispatch
                        uint32_t f;
                        items.get(k, pix, f);
                        next = true;
                        sum = mk(0, 0, 0);
                        fs = f << 16;
                        smp = Sampler{kp.accumulate ? uint32_t(kp.first_frame) + f : 1u,
                                      pcg_hash(items.tx0 + (pix & 7u) + (items.ty0 + (pix >> 3)) * kp.Wu), 0u};
                        ms = MediumStack{0ull, 0};
                    }
#else
                    if ((fs >> 16) < f_end) {  // next frame = next dispatch: statics reset
                        next = true;
                        sum = mk(0, 0, 0);
                        smp.frame = kp.accumulate ? uint32_t(kp.first_frame) + (fs >> 16) : 1u;
                        smp.offset = 0;
                        ms = MediumStack{0ull, 0};
                    }
#endif
                }
                if (!one_sample) s_sum.set(sum);
                if (next) {
#if HG_REGEN_ITEMS
                    const uint32_t qx = items.tx0 + (pix & 7u), qy = items.ty0 + (pix >> 3);
#else
                    const int gtile = kp.rank + local_tile * kp.n_ranks;
                    const uint32_t qx = uint32_t(gtile % kp.tiles_x) * HG_TILE + (pix & 7u);
                    const uint32_t qy = uint32_t(gtile / kp.tiles_x) * HG_TILE + (pix >> 3);
#endif
                    ray = camera_ray(kp, smp, (float(qx) / kp.W) * 2.0f - 1.0f, (float(qy) / kp.H) * 2.0f - 1.0f);
                    thr = mk(1, 1, 1);
                    col = mk(0, 0, 0);
                    acc_rough = 0.0f;
                    bounce = 0;
                    paths++;
                } else {
                    work = false;
                }
            }
            s_thr.set(thr);
            s_col.set(col);
        }
        if (kCounters) {  // t1 was read inside the divergent branch: take it from a lane that ran it
            const uint64_t t2 = wave_clock();
            const int src = __ffsll((unsigned long long)__ballot(was_work)) - 1;
            const uint64_t t1u = (uint64_t(__shfl(uint32_t(t1 >> 32), src)) << 32) | __shfl(uint32_t(t1), src);
            cyc_trav += t1u - t0;
            cyc_shade += t2 - t1u;
        }
    }
    record_tile_cost(lane);
    if (kCounters) {
        const uint32_t v[9] = {paths, c.rays, c.tri, c.aabb, c.rays * uint32_t(kp.n_meshes),
                               c.rays * uint32_t(kp.n_spheres), c.hits, c.node_rounds, c.tri_rounds};
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint32_t sv = wave_sum(v[k]);
            if (lane == 0 && sv) atomicAdd(kp.counters + k, (unsigned long long)sv);
        }
        if (lane == 0) {
            atomicAdd(kp.counters + 9, (unsigned long long)cyc_trav);
            atomicAdd(kp.counters + 10, (unsigned long long)cyc_shade);
        }
        const uint32_t sr = wave_sum(c.shade_rounds);
        if (lane == 0 && sr) atomicAdd(kp.counters + 15, (unsigned long long)sr);
        const uint32_t pm = wave_sum(c.primary_miss);
        if (lane == 0 && pm) atomicAdd(kp.counters + 16, (unsigned long long)pm);
    }
}

// Frame-parallel epilogue: acc = acc*(1-w) + c_f*w for f in frame order (AccumulationShader.shader:33), exactly
// the per-frame blend the kernel does itself when frame_split == 1.
__global__ __launch_bounds__(256) void hg_blend_frames(float4* __restrict__ acc, const float4* __restrict__ colors,
                                                       uint32_t n_slots, int32_t n_frames, int32_t first_frame,
                                                       int32_t accumulate) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_slots) return;
    float4 a = acc[i];
    for (int32_t f = 0; f < n_frames; ++f) {
#if HG_FC_SLOT_MAJOR
        const float4 c = fc_load(colors + size_t(i) * uint32_t(n_frames) + uint32_t(f));  // fc_index (hg_device.h)
#else
        const float4 c = fc_load(colors + size_t(f) * n_slots + i);
#endif
        if (accumulate) {
            const float w = rcp_exact(float(uint32_t(first_frame + f)));
            const float k = 1.0f - w;
            a = make_float4(a.x * k + c.x * w, a.y * k + c.y * w, a.z * k + c.z * w, a.w * k + 1.0f * w);
        } else {
            a = make_float4(c.x, c.y, c.z, 1.0f);
        }
    }
    acc[i] = a;
}

#if HG_FC_SLOT_MAJOR
// The same blend over the [slot][frame] layout: each wave owns 64 slots (a tile) and moves their colours 8 frames at
// a time through LDS, so every load instruction reads whole 128-B lines (8 lanes per line: one slot's 8 frames)
// instead of 64 lanes on 64 lines; then each lane blends its slot's 8 frames in frame order.
__global__ __launch_bounds__(256) void hg_blend_frames_sm(float4* __restrict__ acc, const float4* __restrict__ colors,
                                                          uint32_t n_slots, int32_t n_frames, int32_t first_frame,
                                                          int32_t accumulate) {
    constexpr uint32_t kRow = 9;  // float4 per slot row: 8 frames + 1 pad (spreads the lanes' rows over the banks)
    __shared__ float4 stage[4][64 * kRow];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t slot0 = (blockIdx.x * 4u + w) * 64u;
    if (slot0 >= n_slots) return;  // whole wave: n_slots is a multiple of 64
    const uint32_t nf = uint32_t(n_frames);
    float4* st = stage[w];
    float4 a = acc[slot0 + lane];
    for (uint32_t f0 = 0; f0 < nf; f0 += 8u) {
#pragma unroll
        for (uint32_t r = 0; r < 8u; ++r) {
            const uint32_t j = lane + 64u * r, s = j >> 3, ff = j & 7u;
            if (f0 + ff < nf) st[s * kRow + ff] = fc_load(colors + size_t(slot0 + s) * nf + f0 + ff);
        }
        wave_lds_sync();
        const uint32_t fe = nf - f0 < 8u ? nf - f0 : 8u;
        for (uint32_t ff = 0; ff < fe; ++ff) {
            const float4 c = st[lane * kRow + ff];
            if (accumulate) {
                const float wt = rcp_exact(float(uint32_t(first_frame) + f0 + ff));
                const float k = 1.0f - wt;
                a = make_float4(a.x * k + c.x * wt, a.y * k + c.y * wt, a.z * k + c.z * wt, a.w * k + 1.0f * wt);
            } else {
                a = make_float4(c.x, c.y, c.z, 1.0f);
            }
        }
        wave_lds_sync();
    }
    acc[slot0 + lane] = a;
}
#endif

// The blend of a launch of few frames (at most HG_QUEUE_MAX_FRAMES): one thread per slot, no LDS, 64-thread groups and
// few registers.  A 1-frame launch's blend runs while the next launch's persistent trace waves hold the CUs' wave slots
// and most of their LDS: this one fits beside them (the LDS-staged hg_blend_frames_sm, 36 KB per group, waited for
// the trace to wind down: 0.7 ms per 1-frame blend on C3).  Same operations in the same order.
__global__ __launch_bounds__(64) void hg_blend_frames_lean(float4* __restrict__ acc, const float4* __restrict__ colors,
                                                           uint32_t n_slots, int32_t n_frames, int32_t first_frame,
                                                           int32_t accumulate) {
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= n_slots) return;
    float4 a = acc[i];
    for (int32_t f = 0; f < n_frames; ++f) {
        const float4 c = fc_load(colors + fc_slot_frame(i, uint32_t(f), n_slots, uint32_t(n_frames)));
        if (accumulate) {
            const float w = rcp_exact(float(uint32_t(first_frame + f)));
            const float k = 1.0f - w;
            a = make_float4(a.x * k + c.x * w, a.y * k + c.y * w, a.z * k + c.z * w, a.w * k + 1.0f * w);
        } else {
            a = make_float4(c.x, c.y, c.z, 1.0f);
        }
    }
    acc[i] = a;
}

hipError_t hg_launch_blend_frames(const HgKernelParams& kp, hipStream_t stream) {
    const uint32_t n_slots = uint32_t(kp.n_local_tiles) * 64u;
    if (n_slots == 0) return hipSuccess;
    if (kp.n_frames <= HG_QUEUE_MAX_FRAMES) {
        hipLaunchKernelGGL(hg_blend_frames_lean, dim3((n_slots + 63) / 64), dim3(64), 0, stream, kp.acc, kp.frame_color,
                           n_slots, kp.n_frames, kp.first_frame, kp.accumulate);
        return hipGetLastError();
    }
#if HG_FC_SLOT_MAJOR
    hipLaunchKernelGGL(hg_blend_frames_sm, dim3((n_slots + 255) / 256), dim3(256), 0, stream, kp.acc,
                       kp.frame_color, n_slots, kp.n_frames, kp.first_frame, kp.accumulate);
#else
    hipLaunchKernelGGL(hg_blend_frames, dim3((n_slots + 255) / 256), dim3(256), 0, stream, kp.acc, kp.frame_color,
                       n_slots, kp.n_frames, kp.first_frame, kp.accumulate);
#endif
    return hipGetLastError();
}

// LDS bytes with the mesh records after `base` bytes of rows, or 0 when they do not fit `budget` (or HG_MESH_LDS is off)
static size_t mesh_lds_bytes(size_t base, int32_t n_meshes, size_t budget) {
    if (!HG_MESH_LDS || n_meshes <= 0) return 0;
    const size_t b = base + size_t(n_meshes) * HG_MESH_LDS_F4 * 16u;
    return b <= budget ? b : 0;
}

hipError_t hg_launch_mega_regen(const HgKernelParams& kp_in, int block, bool counters, hipStream_t stream) {
    (void)block;  // one wave per workgroup (the kernel's LDS rows assume it)
    block = 64;
    const int64_t grid = int64_t(kp_in.n_local_tiles) * kp_in.frame_split;
    if (grid == 0) return hipSuccess;
    const uint32_t lds_depth = kp_in.stack_depth < HG_MEGA_LDS_STACK ? kp_in.stack_depth : HG_MEGA_LDS_STACK;
    const size_t lds = size_t(kRegenRowStack + lds_depth) * 64u * sizeof(uint32_t);
    HgKernelParams kp = kp_in;
    kp.mesh_lds_word = uint32_t(lds / 4u);
    const size_t mesh_lds = mesh_lds_bytes(lds, kp.n_meshes, HG_REGEN_LDS_BUDGET);
    const dim3 g{uint32_t(grid)}, b{uint32_t(block)};
    if (counters && mesh_lds) hipLaunchKernelGGL((hg_trace_regen_kernel<true, true>), g, b, mesh_lds, stream, kp);
    else if (counters) hipLaunchKernelGGL((hg_trace_regen_kernel<true, false>), g, b, lds, stream, kp);
    else if (mesh_lds) hipLaunchKernelGGL((hg_trace_regen_kernel<false, true>), g, b, mesh_lds, stream, kp);
    else hipLaunchKernelGGL((hg_trace_regen_kernel<false, false>), g, b, lds, stream, kp);
    return hipGetLastError();
}

// Persistent streaming waves over a work queue (kQueue: launches of at most HG_QUEUE_MAX_FRAMES frames, e.g. the
// reference's one dispatch per frame, RP:327).  The launch has one wave per resident wave slot
// (kp.resident_waves, at most one per unit); each wave pulls (tile, frame chunk) units from the queue and hands their
// (pixel, frame) items to its lanes in order (pixel-major, as TileItems).  A lane that finishes a frame takes the
// wave's next item in place; a lane that finds the current unit spent idles until the top of the wave's loop, where
// the wave pulls the next unit for its idle lanes, while the lanes still on the old unit's items carry on.  So a lane
// idles only between a unit's end and the next loop top, and at the very end of the queue, not until its tile's
// slowest path is done.  Without it a 1-frame launch (one item per pixel) kept each wave's 64 lanes waiting for its
// tile's slowest path: 899 -> 1,383 Mpaths/s on C3 as 1-frame launches.  With 64-frame launches the per-tile waves win
// (one tile's 4,096 items keep the lanes busy anyway; the queue's per-take LDS reads cost C3 2.6 %, C2 6.6 %).  The
// queue is 8 heads, one per XCD
// (workgroups are placed on XCD blockIdx mod 8): head h hands out units h, h + 8, h + 16, ... in the cost order
// (wave_unit), and a wave whose head is dry steals from the others.  Which wave traces an item changes nothing: every
// item runs with the inputs the reference's dispatch of that frame gives its pixel, and writes its own colour slot.
// LDS words read / written by different lanes of the wave: relaxed workgroup-scope atomics on the __shared__ object
// itself compile to plain ds_read / ds_write that the compiler may not cache in registers (a volatile access through
// a cast pointer became a FLAT access with a 64-bit generic address and cost the kernel 60 B of scratch)
constexpr uint32_t kFreshLane = 0xFFFFFFFFu;  // `bounce` of a lane that has no path yet (it takes its item when shading)
// The wave's two current units (double-buffered), in LDS (one wave per workgroup).  Item numbers (hg_next_item) run on
// across units: unit hg_q_cur covers [base, end), the other one the numbers after it, so a lane whose take runs past
// the first unit's items gets the second's at once; the loop top refills the spent unit.
struct QueueUnit {
    uint32_t base, end;                            // the wave's item numbers [base, end) are this unit's items
    uint32_t tile, tx0, ty0, tw, nv, f_begin, nf;  // its tile (local index, origin, width, valid pixels), frames
};
__shared__ QueueUnit hg_qu[2];
__shared__ uint32_t hg_q_cur;  // the unit whose items come first
__shared__ uint32_t hg_q_dry;  // the queue has no unit left
__shared__ uint32_t hg_q_empty;  // the queue has no unit left and both units are spent (the wave's lanes retire)

// Pull the next unit of the queue into hg_qu[slot], its items numbered from `base` (one lane).  When the queue is dry
// the unit is empty (end = base) and hg_q_dry is set.  Attributes the wave clock since the previous pull to the
// previous unit's tile cost (the cost order of the next launches).
__device__ __forceinline__ void queue_pull(const HgKernelParams& kp, uint32_t n_units, uint32_t split, uint32_t slot,
                                           uint32_t base) {
    const uint32_t x = blockIdx.x & 7u;
    uint32_t u = n_units;
    for (uint32_t t = 0; t < 8u && u >= n_units; ++t) {  // own XCD's head first, then steal
        const uint32_t h = (x + t) & 7u;
        if (h >= n_units) continue;
        const uint32_t j = atomicAdd(kp.queue + 32u * h, 1u);
        if (uint64_t(h) + 8ull * j < n_units) u = h + 8u * j;
    }
    QueueUnit& q = hg_qu[slot];
    lds_put(q.base, base);
    if (u >= n_units) {
        lds_put(q.end, base);
        lds_put(hg_q_dry, 1u);
        return;  // the last unit's cost is recorded at the wave's end (record_tile_cost)
    }
    int tile;
    uint32_t chunk;
    wave_unit(kp, u, uint32_t(kp.n_local_tiles), split, tile, chunk);
    const uint32_t fb = uint32_t((uint64_t(chunk) * uint32_t(kp.n_frames)) / split);
    const uint32_t fe = uint32_t((uint64_t(chunk + 1) * uint32_t(kp.n_frames)) / split);
    const uint32_t g = uint32_t(kp.rank) + uint32_t(tile) * uint32_t(kp.n_ranks);
    const uint32_t ty = g / uint32_t(kp.tiles_x);
    const uint32_t tx0 = (g - ty * uint32_t(kp.tiles_x)) * HG_TILE, ty0 = ty * HG_TILE;
    const uint32_t tw = min(uint32_t(HG_TILE), kp.Wu - min(kp.Wu, tx0));
    const uint32_t th = min(uint32_t(HG_TILE), kp.Hu - min(kp.Hu, ty0));
    const uint64_t now = wave_clock();
    unsigned long long* const prev = hg_wave_cost[threadIdx.x >> 6];
    if (prev) cost_add(prev, now - hg_wave_t0[threadIdx.x >> 6]);
    hg_wave_cost[threadIdx.x >> 6] = kp.tile_cost ? kp.tile_cost + tile : nullptr;
    hg_wave_t0[threadIdx.x >> 6] = now;
    lds_put(q.tile, uint32_t(tile));
    lds_put(q.tx0, tx0);
    lds_put(q.ty0, ty0);
    lds_put(q.tw, tw);
    lds_put(q.nv, tw * th);
    lds_put(q.f_begin, fb);
    lds_put(q.nf, fe > fb ? fe - fb : 1u);
    lds_put(q.end, base + tw * th * (fe - fb));
}

// Loop top (lane 0, the whole wave converged): keep both units filled.  Returns true when no item is left anywhere.
__device__ __forceinline__ bool queue_refill(const HgKernelParams& kp, uint32_t n_units, uint32_t split) {
    const uint32_t cnt = lds_get(hg_next_item);
    uint32_t a = lds_get(hg_q_cur);
    if (cnt >= lds_get(hg_qu[a].end) && !lds_get(hg_q_dry)) {  // the first unit is spent
        const uint32_t b = a ^ 1u, b_end = lds_get(hg_qu[b].end);
        if (cnt < b_end) {  // the second one is in use: it comes first now, the spent one is refilled after it
            lds_put(hg_q_cur, b);
            queue_pull(kp, n_units, split, a, b_end);
            a = b;
        } else {  // both spent (numbers taken by lanes that found them so are skipped): two new units
            queue_pull(kp, n_units, split, a, cnt);
            queue_pull(kp, n_units, split, b, lds_get(hg_qu[a].end));
        }
    }
    return lds_get(hg_q_dry) && cnt >= lds_get(hg_qu[a ^ 1u].end) && cnt >= lds_get(hg_qu[a].end);
}

// Item number k of the wave, if one of the two current units holds it: its accumulator slot, frame and pixel
// (pixel-major, as TileItems::get).  Called by the lanes that took k.
__device__ __forceinline__ bool queue_item(uint32_t k, uint32_t& slot, uint32_t& frame, uint32_t& px, uint32_t& py) {
    const uint32_t a = __builtin_amdgcn_readfirstlane(lds_get(hg_q_cur));
    const uint32_t a_end = __builtin_amdgcn_readfirstlane(lds_get(hg_qu[a].end));
    const uint32_t b_end = __builtin_amdgcn_readfirstlane(lds_get(hg_qu[a ^ 1u].end));
    if (k >= b_end && k >= a_end) return false;
    QueueUnit& q = hg_qu[k < a_end ? a : a ^ 1u];
    const uint32_t base = lds_get(q.base);
    if (k < base) return false;  // (never: numbers below the first unit were all handed out before it)
    const uint32_t kk = k - base, nf = lds_get(q.nf), nv = lds_get(q.nv), tw = lds_get(q.tw);
    uint32_t i, f;
    if ((nf & (nf - 1u)) == 0u) {
        const uint32_t lg = uint32_t(__builtin_ctz(nf));
        i = kk >> lg;
        f = kk & (nf - 1u);
    } else {
        i = kk / nf;
        f = kk - i * nf;
    }
    const uint32_t pix = nv == 64u ? i : (i % tw) + 8u * (i / tw);
    slot = lds_get(q.tile) * 64u + pix;
    frame = lds_get(q.f_begin) + f;
    px = lds_get(q.tx0) + (pix & 7u);
    py = lds_get(q.ty0) + (pix >> 3);
    return true;
}

// The lanes calling it (the active lanes) take the wave's next item numbers in lane order (one LDS atomic)
__device__ __forceinline__ uint32_t queue_take() {
    const uint64_t m = __builtin_amdgcn_read_exec();
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
    uint32_t b0 = 0;
    if (rank == 0u) b0 = atomicAdd(&hg_next_item, uint32_t(__builtin_popcountll(m)));
    return __builtin_amdgcn_readfirstlane(b0) + rank;
}

// The image pixel of accumulator slot `slot` (local tile slot / 64, pixel slot % 64)
__device__ __forceinline__ void slot_pixel(const HgKernelParams& kp, uint32_t slot, uint32_t& x, uint32_t& y) {
    const uint32_t g = uint32_t(kp.rank) + (slot >> 6) * uint32_t(kp.n_ranks);
    const uint32_t ty = g / uint32_t(kp.tiles_x);
    x = (g - ty * uint32_t(kp.tiles_x)) * HG_TILE + (slot & 7u);
    y = ty * HG_TILE + ((slot >> 3) & 7u);
}

#if HG_MIG_KERNEL
// Path migration (kQueue).  After the queue runs dry each wave drains: its lanes finish the paths they
// hold, the idle ones waiting, the wave's slot held until its slowest path ends.  Here a dry wave with at most
// HG_MIG_RETIRE paths left retires: each of its lanes, when its current ray ends and the path goes on, writes the
// path's whole state (a ray boundary: no traversal state) to a pool record instead of beginning the ray, and the wave
// leaves once its lanes are empty; the dry waves that stay take pool records into their idle lanes at the loop top.
// A path's result does not depend on which lane traces it (the state moves bit for bit).  The 64-bit state word counts
// the waves gone (retired or left) and, above bit 32, the retired waves still exporting: a wave retires only while
// another wave of the launch is not gone, and the last one leaves only with no exporter left and the pool empty, so
// every record is taken.  Records carry slot + 1 as their ready flag (0: not written yet), cleared by the taker.
__device__ __forceinline__ uint32_t mig_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Device-coherent single words (relaxed agent-scope atomics: written through to / read from the coherent level).  No
// acquire / release fences: at agent scope on gfx950 those write back or invalidate the XCD's whole L2, and one per
// wave leaving made 1-frame launches 2x slower (the waves lost their cached nodes); mig_drain orders a lane's stores.
__device__ __forceinline__ void mig_st(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void mig_drain() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ unsigned long long* mig_state(const HgKernelParams& kp) {
    return reinterpret_cast<unsigned long long*>(kp.queue + HG_MIG_STATE_WORD);
}
__device__ __forceinline__ uint4* mig_rec(const HgKernelParams& kp, uint32_t i) {
    return reinterpret_cast<uint4*>(reinterpret_cast<char*>(kp.queue) + HG_MIG_POOL_BYTE) + 8u * i;
}
// the pool's counts in one 64-bit word: records reserved (low half) and taken (high half), one load to test it
__device__ __forceinline__ unsigned long long* mig_pool(const HgKernelParams& kp) {
    return reinterpret_cast<unsigned long long*>(kp.queue + HG_MIG_POOL_WORD);
}
__device__ __forceinline__ bool mig_pool_empty(const HgKernelParams& kp) {
    const unsigned long long v = __hip_atomic_load(mig_pool(kp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return uint32_t(v >> 32) >= uint32_t(v);
}
// lane 0: retire the wave, unless the pool holds records to take or it would leave fewer than gridDim >> HG_MIG_KEEP_SHIFT
// waves of the launch not gone (at least one)
__device__ __forceinline__ bool mig_try_retire(const HgKernelParams& kp) {
    if (!mig_pool_empty(kp)) return false;
    unsigned long long* const s = mig_state(kp);
    unsigned long long v = __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int t = 0; t < 16; ++t) {
        if (uint32_t(v) + 1u + (gridDim.x >> HG_MIG_KEEP_SHIFT) > gridDim.x || uint32_t(v) + 1u >= gridDim.x) return false;
        if (__hip_atomic_compare_exchange_strong(s, &v, v + 1ull + (1ull << 32), __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return true;
    }
    return false;
}
// lane 0 of a wave with no path: leave, if the pool is empty and either another wave is not gone or no retired wave
// is still exporting (a successful exchange of the word read proves no wave retired since)
__device__ __forceinline__ bool mig_try_leave(const HgKernelParams& kp) {
    unsigned long long* const s = mig_state(kp);
    unsigned long long v = __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int t = 0; t < 16; ++t) {
        if (uint32_t(v) + 1u >= gridDim.x && (v >> 32) != 0ull) return false;
        if (!mig_pool_empty(kp)) return false;
        if (__hip_atomic_compare_exchange_strong(s, &v, v + 1ull, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return true;
    }
    return false;
}
// lane 0: claim up to `want` pool records (first in `first`)
__device__ __forceinline__ uint32_t mig_claim(const HgKernelParams& kp, uint32_t want, uint32_t& first) {
    unsigned long long* const pool = mig_pool(kp);
    unsigned long long v = __hip_atomic_load(pool, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int t = 0; t < 16; ++t) {
        const uint32_t p = uint32_t(v), q = uint32_t(v >> 32);
        if (q >= p) return 0u;
        const uint32_t n = min(want, p - q);
        if (__hip_atomic_compare_exchange_strong(pool, &v, v + (uint64_t(n) << 32), __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
            first = q;
            return n;
        }
    }
    return 0u;
}
#endif

#ifndef HG_RAY_SORT
#define HG_RAY_SORT 0  // A/B (DESIGN.md §10 lever 7): 1 = sort the lanes beginning a ray by direction octant, 2 = by
                       // octant and dominant axis (24 keys), before their traversal
#endif
#if HG_RAY_SORT
// Ray-coherence experiment.  A vector load costs the texture-data unit per distinct cache line in each 16-lane quarter
// of the wave, not per line of the whole wave (tools/micro_lane_order.hip: 4 lines per instruction cost 19 cycles with
// each line's lanes in one quarter and 51-65 with them spread), so rays that visit the same nodes should sit in the same
// quarter.  The lanes that begin a ray in a shading pass (`began`) exchange their whole path state so that equal sort
// keys are adjacent: a counting sort of the keys by ballots; lane l writes its own lane number to LDS word pos(l) of the
// scratch row; the began lane of rank r among the began lanes reads word r, the lane whose state it takes; every state
// word moves by ds_bpermute (full EXEC: the other lanes take their own).  Which lane runs a path changes no result.
__device__ __forceinline__ uint32_t ray_key(const f3& d) {
    const uint32_t oct = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
#if HG_RAY_SORT == 2
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    const uint32_t dom = ax >= ay && ax >= az ? 0u : ay >= az ? 1u : 2u;
    return oct * 3u + dom;
#else
    return oct;
#endif
}
constexpr uint32_t kRayKeys = HG_RAY_SORT == 2 ? 24u : 8u;
__device__ __forceinline__ uint32_t bperm(uint32_t src, uint32_t v) {
    return uint32_t(__builtin_amdgcn_ds_bpermute(int(src << 2), int(v)));
}
__device__ __forceinline__ float bpermf(uint32_t src, float v) { return __uint_as_float(bperm(src, __float_as_uint(v))); }
#endif

// Streaming variant (HG_KERNEL_MEGA_STREAM): the regenerating kernel with a resumable traversal.  Lanes advance
// their traversal one while-while round at a time; once at most HG_STREAM_TMIN lanes are still traversing (and
// some have finished), the finished lanes shade their hit and start their next ray while the stragglers keep
// their traversal state, so the wave's lanes stay busy instead of waiting for the slowest ray of every bounce.
// Every frame's colour goes to frame_color (item scheduling), blended in frame order by hg_blend_frames.  kQueue: the
// persistent work-queue form above (launches of few frames).
template <bool kCounters, bool kMeshLds, bool kQueue, bool kDeep>
__global__ __launch_bounds__(HG_STREAM_LB, HG_STREAM_WAVES) void hg_trace_stream_kernel(const HgKernelParams kp) {
    // shade once at most kTmin lanes still traverse; reshade while at least kReshade need it (compile-time: as kernel
    // parameters they cost 8 B of scratch)
    constexpr uint32_t kTmin = kDeep ? HG_STREAM_TMIN_DEEP : HG_STREAM_TMIN;
    constexpr uint32_t kReshade = kDeep ? HG_STREAM_RESHADE_DEEP : HG_STREAM_RESHADE;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nlt = uint32_t(kp.n_local_tiles), split = uint32_t(kp.frame_split);
    const uint32_t n_units = nlt * split;  // kQueue: (tile, frame chunk) units of the queue
    int local_tile = 0;
    uint32_t chunk = 0, f_begin = 0, f_end = 0, u_first = 0;
    if constexpr (kQueue) {
        if (lane == 0) {
            lds_put(hg_next_item, 0u);
            for (uint32_t u = 0; u < 2u; ++u) {
                lds_put(hg_qu[u].base, 0u);
                lds_put(hg_qu[u].end, 0u);
            }
            lds_put(hg_q_cur, 0u);
            lds_put(hg_q_dry, 0u);
            hg_wave_cost[threadIdx.x >> 6] = nullptr;
        }
    } else {
        // wave -> (tile, frame chunk), as in hg_trace_regen_kernel
        // one wave per workgroup (launched with 64 threads): wave = workgroup
        const uint32_t gw = xcd_block(blockIdx.x, gridDim.x);
        u_first = gw * (kp.wave_units > 1u ? kp.wave_units : 1u);  // (more than one unit only without a frame split)
        wave_unit(kp, u_first, nlt, split, local_tile, chunk);
        tile_cost_begin(kp, lane, local_tile, chunk < split);
        f_begin = uint32_t((uint64_t(chunk) * uint32_t(kp.n_frames)) / split);
        f_end = uint32_t((uint64_t(chunk + 1) * uint32_t(kp.n_frames)) / split);
    }
    const RowStack<HG_STREAM_LDS_STACK, kRowStack> stk{lane, kp.spill + blockIdx.x * 64u + lane, kp.spill_stride};
    const RowVec3<kRowThr> s_thr{lane};
    const RowVec3<kRowCol> s_col{lane};
    const RowVec3<kRowSum> s_sum{lane};
    const LeafShare ls{kRowLeaf * 64u};
    const uint32_t nm = uint32_t(kp.n_meshes);
    if (kMeshLds) {  // the wave's copy of the mesh records (mesh_f4, hg_device.h)
        mesh_lds_fill(kp, lane);
        wave_lds_sync();
    }
#if HG_NODE_CACHE
    {  // the wave's copy of the hot node records (written before any lane reads it: one wave per workgroup)
        float4* cache = reinterpret_cast<float4*>(hg_lds_stack + kRowCache * 64u);
        const uint32_t nf4 = 4u * (kp.hot_records < HG_NODE_CACHE ? kp.hot_records : uint32_t(HG_NODE_CACHE));
        for (uint32_t i = lane; i < nf4; i += 64u) cache[i] = kp.nodes[i];
        wave_lds_sync();
    }
#endif
#if HG_WAVE_TIMELINE
    uint64_t tl_start = 0, tl_dry = 0;
    if (kQueue && kp.timeline) tl_start = __builtin_amdgcn_s_memrealtime();
#endif
    bool work = false;
    uint32_t px = 0u, py = 0u;
    Counters c{0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t paths = 0;
    uint32_t fs = f_begin << 16;  // frame index << 16 | sample index
    uint32_t bounce = 0;          // diffuse | glossy << 8 | transmission << 16 | bounce index << 24
    Sampler smp{kp.accumulate ? uint32_t(kp.first_frame) + f_begin : 1u, pcg_hash(px + py * kp.Wu), 0u};
    MediumStack ms{0ull, 0};
    Ray ray{mk(0, 0, 0), mk(0, 0, 1)};
    float acc_rough = 0.0f;
    Trav tv;
    tv.mi = nm;
    uint32_t slot = 0;  // the lane's item: kQueue its accumulator slot (local tile * 64 + pixel), else v (UnitItems)
    bool dry = false;   // kQueue, wave-uniform: the queue has no unit left
#if HG_MIG_KERNEL
    // (kQueue, wave-uniform) 1: the wave exports its paths at their ray boundaries, then leaves.  The kernel is at
    // its scalar-register limit: every wave-uniform value live across the loop spills (a lane holding an imported
    // path is marked by its mesh cursor, tv.mi = nm + 1, not by a mask)
    uint32_t retiring = 0;
#endif
    const UnitItems items = kQueue ? UnitItems() : UnitItems(kp, u_first, local_tile, chunk < split, f_begin, f_end, lane);
    if constexpr (kQueue) {
        wave_lds_sync();  // hg_q / hg_next_item initialised (lane 0); every lane takes its first item in the loop
    } else {
        if (lane < items.n_items) {  // item `lane`
            uint32_t f;
            items.get(kp, lane, slot, f);
            items.pixel(slot, px, py);
            fs = f << 16;
            smp = Sampler{kp.accumulate ? uint32_t(kp.first_frame) + f : 1u, pcg_hash(px + py * kp.Wu), 0u};
        }
        work = lane < items.n_items;
        if (work) {
            ray = camera_ray(kp, smp, (float(px) / kp.W) * 2.0f - 1.0f, (float(py) / kp.H) * 2.0f - 1.0f);  // :1023-1033
            paths++;
            s_thr.set(mk(1, 1, 1));
            s_col.set(mk(0, 0, 0));
            s_sum.set(mk(0, 0, 0));
            trav_begin<kMeshLds>(kp, ray, tv, c);
        }
    }
    uint64_t cyc_trav = 0, cyc_shade = 0;  // wave clock (s_memtime) per phase, counting instantiation only
#if HG_DRAIN_PRIO
    __builtin_amdgcn_s_setprio(2);
#elif HG_SHADE_PRIO >= 2
    __builtin_amdgcn_s_setprio(HG_SHADE_PRIO - 1);  // traversal waits on memory: its waves issue first
#endif
    for (;;) {
        // ---- kQueue: the wave refills a spent unit, and idle lanes (the wave's start; lanes whose take found both
        // units spent) become fresh: they take their item in the shading pass below
        if (kQueue && !dry) {
            wave_lds_sync();
            if (lane == 0u) lds_put(hg_q_empty, queue_refill(kp, n_units, split) ? 1u : 0u);
            wave_lds_sync();
            dry = __builtin_amdgcn_readfirstlane(lds_get(hg_q_empty)) != 0u;
#if HG_WAVE_TIMELINE
            if (dry && kp.timeline) tl_dry = __builtin_amdgcn_s_memrealtime();
#endif
            if (!work && !dry) {
                work = true;
                bounce = kFreshLane;
                tv.mi = nm;
            }
        }
#if HG_MIG_KERNEL
        if (kQueue && dry) {  // (the whole wave converged)
            if (retiring) {
                if (!__any(work)) {  // every path exported or finished
                    mig_drain();  // (the wave's records are flagged before it stops counting as exporting)
                    if (lane == 0u)
                        __hip_atomic_fetch_add(mig_state(kp), 0xFFFFFFFF00000000ull, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            } else {
                // idle lanes take exported paths (their state as the exporting lane left it at a ray boundary)
                // (each test of the pool is a device-coherent load, microseconds: a wave with most lanes busy tests it
                // every HG_MIG_POLL-th loop only)
                bool leave_now = false, poll = false;
                uint32_t mig_spins = 0;
                for (;;) {  // (an inner loop: a second latch of the outer loop cost the kernel scratch)
                const uint64_t idle = wave_ballot(!work);
                const uint32_t n_idle = uint32_t(__builtin_popcountll(idle));
                poll = n_idle >= uint32_t(HG_MIG_POLL_IDLE);
                uint32_t n = 0, q0 = 0;
                if (poll && lane == 0u) n = mig_claim(kp, n_idle, q0);
                n = __builtin_amdgcn_readfirstlane(n);
                q0 = __builtin_amdgcn_readfirstlane(q0);
                const uint32_t r = __builtin_amdgcn_mbcnt_hi(uint32_t(idle >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(idle), 0u));
                if (!work && r < n) {
                    uint4* const rec = mig_rec(kp, q0 + r);
                    uint32_t* const flag = &rec[6].x;
                    uint32_t s1 = mig_ld(flag);
                    for (uint32_t k = 0; s1 == 0u && k < (1u << 22); ++k) {  // (reserved: its writer is resident)
                        __builtin_amdgcn_s_sleep(1);
                        s1 = mig_ld(flag);
                    }
                    const uint32_t* const w = reinterpret_cast<const uint32_t*>(rec);
                    ray.o = mk(__uint_as_float(mig_ld(w + 0)), __uint_as_float(mig_ld(w + 1)), __uint_as_float(mig_ld(w + 2)));
                    ray.d = mk(__uint_as_float(mig_ld(w + 3)), __uint_as_float(mig_ld(w + 4)), __uint_as_float(mig_ld(w + 5)));
                    s_thr.set(mk(__uint_as_float(mig_ld(w + 6)), __uint_as_float(mig_ld(w + 7)), __uint_as_float(mig_ld(w + 8))));
                    s_col.set(mk(__uint_as_float(mig_ld(w + 9)), __uint_as_float(mig_ld(w + 10)), __uint_as_float(mig_ld(w + 11))));
                    acc_rough = __uint_as_float(mig_ld(w + 12));
                    fs = mig_ld(w + 13);
                    bounce = mig_ld(w + 14);
                    smp.frame = mig_ld(w + 15);
                    smp.pixel = mig_ld(w + 16);
                    smp.offset = mig_ld(w + 17);
                    ms.s = uint64_t(mig_ld(w + 18)) | (uint64_t(mig_ld(w + 19)) << 32);
                    ms.sp = int(mig_ld(w + 20));
                    __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    slot = s1 - 1u;
                    work = true;
                    tv.mi = nm + 1u;  // waits to shade: the shading pass begins its ray
                }
                if (__any(work)) break;
                uint32_t leave = 0;
                if (lane == 0u) leave = mig_try_leave(kp) ? 1u : 0u;
                if (__builtin_amdgcn_readfirstlane(leave) || ++mig_spins >= (1u << 22)) {
                    leave_now = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(4);  // the launch's last wave: exporters are still at work
                }
                if (leave_now) break;
                if (poll && kp.spp == 1 && wave_count(work) <= uint32_t(HG_MIG_RETIRE)) {  // (a sample sum stays)
                    uint32_t ret = 0;
                    if (lane == 0u) ret = mig_try_retire(kp) ? 1u : 0u;
                    retiring = __builtin_amdgcn_readfirstlane(ret);
                }
            }
        }
#endif
        if (!__any(work)) break;
        // ---- traversal rounds until few lanes are left traversing
        if (kCounters) cyc_trav -= wave_clock();
        for (;;) {
            const bool act = work && tv.mi < nm;
            const uint64_t am = wave_ballot(act);
            // (work includes act: some lane waits to shade iff the work mask differs)
            if (am == 0ull || (uint32_t(__builtin_popcountll(am)) <= kTmin && wave_ballot(work) != am)) break;
            trav_step<kMeshLds>(kp, ray, tv, c, stk, act, ls);
        }
        if (kCounters) {
            const uint64_t t = wave_clock();
            cyc_trav += t;
            cyc_shade -= t;
        }
#if HG_DRAIN_PRIO  // (A/B) a queue wave past its queue's end drains at the lowest priority in both phases
        if (kQueue && dry) __builtin_amdgcn_s_setprio(0);
        else __builtin_amdgcn_s_setprio(1);
#elif HG_SHADE_PRIO == 1
        __builtin_amdgcn_s_setprio(1);
#elif HG_SHADE_PRIO >= 2
        __builtin_amdgcn_s_setprio(0);
#endif
        // ---- finished lanes: shade, then start their next ray (a ray with nothing to traverse shades again)
        // (rays that finish at once — everything culled — shade again in this loop while at least
        // HG_STREAM_RESHADE lanes need it, otherwise in the next shading phase)
        for (uint32_t it = 0;; ++it) {
            const uint32_t n_sh = wave_count(work && tv.mi >= nm);
            if (n_sh == 0u || (it > 0u && n_sh < kReshade)) break;
#if HG_RAY_SORT
            bool began = false;  // this lane begins a ray (its traversal starts after the sort below)
#endif
            if (work && tv.mi >= nm) {
            c.shade_rounds += wave_once();
#if HG_PHASE_DETAIL == 1
            uint64_t tp = kCounters ? wave_clock() : 0;
#endif
            const bool fresh = kQueue && bounce == kFreshLane;  // no path yet: straight to the take below
#if HG_MIG_KERNEL
            const bool imported = kQueue && tv.mi == nm + 1u;  // begin the imported path's ray
#else
            constexpr bool imported = false;
#endif
            bool alive = imported;
            f3 thr = s_thr.get(), col = s_col.get();
            if (!fresh && !imported) {
            const Hit hit = trav_hit<kMeshLds>(kp, ray, tv);
#if HG_PHASE_DETAIL == 1
            if (kCounters) tp = phase_mark(kp, 11, tp);
#endif
            if (hit.t < kp.far_) {  // :898-936
                c.hits++;
                const Mat mt = load_mat(kp, hit.mat);
                col = col + xyz(mt.emis_rough) * thr;
                uint32_t bt = 0;
                const f3 att = evaluate_hit(kp, smp, ms, ray, hit, mt, bt);
                bounce += 1u << (8u * bt);
                thr = thr * att;
                acc_rough += mt.emis_rough.w * thr.x;
                const float rr = smp.get1(ID_RR);
                smp.offset += BOUNCE_INC;
                const float contribution = fmaxf(fmaxf(thr.x, thr.y), thr.z);
                if (!(rr > contribution)) {
                    thr = thr * rcp_exact(contribution);
                    bounce += 1u << 24;
                    alive = (bounce >> 24) <= kp.max_bounces && !((bounce & 0xFFu) > kp.max_diff ||
                                                                 ((bounce >> 8) & 0xFFu) > kp.max_glossy ||
                                                                 ((bounce >> 16) & 0xFFu) > kp.max_trans);
                }
            } else {  // :941
                c.primary_miss += bounce == 0u;  // the path's camera ray (no bounce recorded yet)
                col = col + sample_sky(kp, ray.d, sky_level(kp, acc_rough)) * thr;
            }
            }
#if HG_PHASE_DETAIL == 1
            if (kCounters) tp = phase_mark(kp, 12, tp);
#endif
            if (!alive) {
                // RayColor += trace_ray(...); spp 1: the sum is the path's colour (0 + col == col bit for bit: col
                // is never -0, it starts at +0 and only has terms added)
                const bool one_sample = kp.spp == 1;
                f3 sum = one_sample ? col : s_sum.get() + col;
                ++fs;
                bool next = !fresh && (fs & 0xFFFFu) < kp.spp;  // next sample: statics persist (:188-189)
                if (!next) {
                    const f3 color = sample_mean(kp, sum);
                    const size_t slot_i = kQueue ? size_t(slot) : size_t(items.slot(slot));
                    // this frame's colour, blended later in frame order (hg_blend_frames)
#if !HG_DIAG_NO_FC  // (analysis builds only: the write-traffic attribution of DESIGN.md §4.5)
                    if (!fresh)
                        fc_store(kp.frame_color + fc_index(kp, fs >> 16, slot_i), make_float4(color.x, color.y, color.z, 1.0f));
#endif
                    fs = (fs & 0xFFFF0000u) + 0x10000u;
                    if constexpr (kQueue) {
                        uint32_t f = 0, hx = 0, hy = 0;
                        if (queue_item(queue_take(), slot, f, hx, hy)) {  // the unit's next item: statics reset
                            next = true;
                            sum = mk(0, 0, 0);
                            fs = f << 16;
                            smp = Sampler{kp.accumulate ? uint32_t(kp.first_frame) + f : 1u, pcg_hash(hx + hy * kp.Wu),
                                          0u};
                            ms = MediumStack{0ull, 0};
                        }
                    } else {
                        const uint32_t k = items.take_here();
                        if (k < items.n_items) {  // the next (pixel, frame) item: statics reset as for a dispatch
                            uint32_t f, hx, hy;
                            items.get(kp, k, slot, f);
                            items.pixel(slot, hx, hy);
                            next = true;
                            sum = mk(0, 0, 0);
                            fs = f << 16;
                            smp = Sampler{kp.accumulate ? uint32_t(kp.first_frame) + f : 1u, pcg_hash(hx + hy * kp.Wu),
                                          0u};
                            ms = MediumStack{0ull, 0};
                        }
                    }
                }
                if (!one_sample) s_sum.set(sum);
                if (next) {
                    {
                        uint32_t qx, qy;
                        if constexpr (kQueue) slot_pixel(kp, slot, qx, qy);
                        else items.pixel(slot, qx, qy);
                        ray = camera_ray(kp, smp, (float(qx) / kp.W) * 2.0f - 1.0f, (float(qy) / kp.H) * 2.0f - 1.0f);
                    }
                    thr = mk(1, 1, 1);
                    col = mk(0, 0, 0);
                    acc_rough = 0.0f;
                    bounce = 0;
                    paths++;
                    alive = true;
                } else {
                    work = false;
                }
            }
            s_thr.set(thr);
            s_col.set(col);
#if HG_PHASE_DETAIL == 1
            if (kCounters) tp = phase_mark(kp, 13, tp);
#endif
#if HG_MIG_KERNEL
            if (kQueue && retiring && alive) {  // export the path at its ray boundary (taken by a staying wave)
                const uint64_t m = __builtin_amdgcn_read_exec();
                const uint32_t rk = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
                uint32_t b0 = 0;
                if (rk == 0u) b0 = uint32_t(atomicAdd(mig_pool(kp), (unsigned long long)__builtin_popcountll(m)));
                uint4* const rec = mig_rec(kp, __builtin_amdgcn_readfirstlane(b0) + rk);
                uint32_t* const w = reinterpret_cast<uint32_t*>(rec);
                const uint32_t v[21] = {__float_as_uint(ray.o.x), __float_as_uint(ray.o.y), __float_as_uint(ray.o.z),
                                        __float_as_uint(ray.d.x), __float_as_uint(ray.d.y), __float_as_uint(ray.d.z),
                                        __float_as_uint(thr.x), __float_as_uint(thr.y), __float_as_uint(thr.z),
                                        __float_as_uint(col.x), __float_as_uint(col.y), __float_as_uint(col.z),
                                        __float_as_uint(acc_rough), fs, bounce, smp.frame, smp.pixel, smp.offset,
                                        uint32_t(ms.s), uint32_t(ms.s >> 32), uint32_t(ms.sp)};
#pragma unroll
                for (int k = 0; k < 21; ++k) mig_st(w + k, v[k]);
                mig_drain();  // the record's words are out before its flag
                mig_st(w + 24, slot + 1u);
                alive = false;
                work = false;
            }
#endif
#if HG_RAY_SORT
            began = alive;
#else
            if (alive) trav_begin<kMeshLds>(kp, ray, tv, c);
#endif
#if HG_PHASE_DETAIL == 1
            if (kCounters) tp = phase_mark(kp, 14, tp);
#endif
            }
#if HG_RAY_SORT
            {  // converged: permute the began lanes' path states into key order, then begin their traversals
                const uint64_t bm = wave_ballot(began);
                if (__builtin_popcountll(bm) >= 2) {
                    const uint32_t key = began ? ray_key(ray.d) : kRayKeys;
                    uint32_t pos = 0, base = 0;
                    for (uint32_t v = 0; v < kRayKeys; ++v) {
                        const uint64_t m = wave_ballot(key == v);
                        if (key == v)
                            pos = base + __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
                        base += uint32_t(__builtin_popcountll(m));
                    }
                    uint32_t* const scratch = hg_lds_stack + kRowSort * 64u;
                    if (began) scratch[pos] = lane;
                    wave_lds_sync();
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi(uint32_t(bm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(bm), 0u));
                    const uint32_t src = began ? scratch[rank] : lane;
                    wave_lds_sync();
                    ray.o = mk(bpermf(src, ray.o.x), bpermf(src, ray.o.y), bpermf(src, ray.o.z));
                    ray.d = mk(bpermf(src, ray.d.x), bpermf(src, ray.d.y), bpermf(src, ray.d.z));
                    fs = bperm(src, fs);
                    bounce = bperm(src, bounce);
                    smp.frame = bperm(src, smp.frame);
                    smp.pixel = bperm(src, smp.pixel);
                    smp.offset = bperm(src, smp.offset);
                    ms.s = (uint64_t(bperm(src, uint32_t(ms.s >> 32))) << 32) | bperm(src, uint32_t(ms.s));
                    ms.sp = int(bperm(src, uint32_t(ms.sp)));
                    acc_rough = bpermf(src, acc_rough);
                    slot = bperm(src, slot);
                    const RowVec3<kRowThr> o_thr{src};
                    const RowVec3<kRowCol> o_col{src};
                    const f3 t_thr = o_thr.get(), t_col = o_col.get();
                    f3 t_sum = mk(0, 0, 0);
                    if (kp.spp != 1) t_sum = RowVec3<kRowSum>{src}.get();
                    wave_lds_sync();
                    s_thr.set(t_thr);
                    s_col.set(t_col);
                    if (kp.spp != 1) s_sum.set(t_sum);
                    wave_lds_sync();
                }
                if (began) trav_begin<kMeshLds>(kp, ray, tv, c);
            }
#endif
        }
#if HG_DRAIN_PRIO
        if (kQueue && dry) __builtin_amdgcn_s_setprio(0);
        else __builtin_amdgcn_s_setprio(2);
#elif HG_SHADE_PRIO == 1
        __builtin_amdgcn_s_setprio(0);
#elif HG_SHADE_PRIO >= 2
        __builtin_amdgcn_s_setprio(HG_SHADE_PRIO - 1);
#endif
        if (kCounters) cyc_shade += wave_clock();
    }
    if constexpr (kQueue) record_tile_cost(lane);
    else items.record_cost(kp, lane);
#if HG_WAVE_TIMELINE
    if (kQueue && kp.timeline && lane == 0u && blockIdx.x < HG_TIMELINE_WAVES) {
        unsigned long long* const w = kp.timeline + 4u * blockIdx.x;
        w[0] = tl_start;
        w[1] = tl_dry;
        w[2] = __builtin_amdgcn_s_memrealtime();
        w[3] = lds_get(hg_next_item);
    }
#endif
    if constexpr (kQueue) {
        // The last wave out resets the queue heads for the next launch on this stream (no memset launch per queue
        // launch: a blit kernel waited for a CU that the other streams' persistent waves held).  A wave leaves only
        // once its pulls found the queue dry, and it pulls no more after that: every head access of the launch
        // happens before the last wave's increment of the exit count (release / acquire).
        if (lane == 0u) {
#if HG_QUEUE_DONE_RELAXED  // (A/B) the head atomics all returned before each wave's increment: no L2 write-back /
                           // invalidate of the XCD per wave leaving
            const uint32_t out = __hip_atomic_fetch_add(kp.queue + HG_QUEUE_DONE_WORD, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
#else
            const uint32_t out = __hip_atomic_fetch_add(kp.queue + HG_QUEUE_DONE_WORD, 1u, __ATOMIC_ACQ_REL,
                                                        __HIP_MEMORY_SCOPE_AGENT);
#endif
            if (out == gridDim.x - 1u) {
                for (uint32_t h = 0; h < 8u; ++h)
                    __hip_atomic_store(kp.queue + 32u * h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if HG_MIG_KERNEL
                __hip_atomic_store(mig_state(kp), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(mig_pool(kp), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
                __hip_atomic_store(kp.queue + HG_QUEUE_DONE_WORD, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (kCounters) {
        const uint32_t v[9] = {paths, c.rays, c.tri, c.aabb, c.rays * nm, c.rays * uint32_t(kp.n_spheres), c.hits,
                               c.node_rounds, c.tri_rounds};
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint32_t sv = wave_sum(v[k]);
            if (lane == 0 && sv) atomicAdd(kp.counters + k, (unsigned long long)sv);
        }
        if (lane == 0) {
            atomicAdd(kp.counters + 9, (unsigned long long)cyc_trav);
            atomicAdd(kp.counters + 10, (unsigned long long)cyc_shade);
        }
        const uint32_t sr = wave_sum(c.shade_rounds);
        if (lane == 0 && sr) atomicAdd(kp.counters + 15, (unsigned long long)sr);
        const uint32_t pm = wave_sum(c.primary_miss);
        if (lane == 0 && pm) atomicAdd(kp.counters + 16, (unsigned long long)pm);
    }
}

hipError_t hg_launch_mega_stream(const HgKernelParams& kp_in, int block, bool counters, hipStream_t stream) {
    (void)block;  // one wave per workgroup (the kernel's LDS rows assume it)
    int64_t grid = int64_t(kp_in.n_local_tiles) * kp_in.frame_split;
    const bool queue = kp_in.queue != nullptr;  // the runtime passes a queue for launches of few frames
    if (queue) grid = grid < int64_t(kp_in.resident_waves) ? grid : int64_t(kp_in.resident_waves);  // persistent waves
    else if (kp_in.wave_units > 1u && kp_in.frame_split == 1)  // wave_units tiles per wave (UnitItems)
        grid = (grid + kp_in.wave_units - 1) / kp_in.wave_units;
    if (grid == 0) return hipSuccess;
    const uint32_t lds_depth = kp_in.stack_depth < HG_STREAM_LDS_STACK ? kp_in.stack_depth : HG_STREAM_LDS_STACK;
    const size_t lds = size_t(kRowStack + lds_depth) * 64u * sizeof(uint32_t) + HG_STREAM_LDS_PAD;
    HgKernelParams kp = kp_in;
    kp.mesh_lds_word = uint32_t(lds / 4u);
    const size_t mesh_lds = mesh_lds_bytes(lds, kp.n_meshes, HG_WAVE_LDS_BUDGET);
    const dim3 g{uint32_t(grid)}, b{64u};
    const size_t sh = mesh_lds ? mesh_lds : lds;
    // deep BLAS (kp.stream_deep): the kDeep thresholds
#define HG_STREAM_LAUNCH(C, M, Q)                                                                                      \
    do {                                                                                                               \
        if (kp.stream_deep) hipLaunchKernelGGL((hg_trace_stream_kernel<C, M, Q, true>), g, b, sh, stream, kp);        \
        else hipLaunchKernelGGL((hg_trace_stream_kernel<C, M, Q, false>), g, b, sh, stream, kp);                      \
    } while (0)
    if (queue) {
        if (counters && mesh_lds) HG_STREAM_LAUNCH(true, true, true);
        else if (counters) HG_STREAM_LAUNCH(true, false, true);
        else if (mesh_lds) HG_STREAM_LAUNCH(false, true, true);
        else HG_STREAM_LAUNCH(false, false, true);
    } else {
        if (counters && mesh_lds) HG_STREAM_LAUNCH(true, true, false);
        else if (counters) HG_STREAM_LAUNCH(true, false, false);
        else if (mesh_lds) HG_STREAM_LAUNCH(false, true, false);
        else HG_STREAM_LAUNCH(false, false, false);
    }
#undef HG_STREAM_LAUNCH
    return hipGetLastError();
}

// Launcher used by the runtime (hg_runtime.hip)
hipError_t hg_launch_mega(const HgKernelParams& kp, int block, bool counters, hipStream_t stream) {
    const int tiles_per_block = block / 64;
    const int grid = (kp.n_local_tiles + tiles_per_block - 1) / tiles_per_block;
    if (grid == 0) return hipSuccess;
    const size_t lds = hg_mega_lds_bytes(kp.stack_depth, block);
    const bool dbg = kp.debug_mode != 0;
    if (counters && dbg)
        hipLaunchKernelGGL((hg_trace_kernel<true, true>), dim3(uint32_t(grid)), dim3(block), lds, stream, kp);
    else if (counters)
        hipLaunchKernelGGL((hg_trace_kernel<true, false>), dim3(uint32_t(grid)), dim3(block), lds, stream, kp);
    else if (dbg)
        hipLaunchKernelGGL((hg_trace_kernel<false, true>), dim3(uint32_t(grid)), dim3(block), lds, stream, kp);
    else
        hipLaunchKernelGGL((hg_trace_kernel<false, false>), dim3(uint32_t(grid)), dim3(block), lds, stream, kp);
    return hipGetLastError();
}
