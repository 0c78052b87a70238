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
    const int local_tile = int(blockIdx.x) * int(blockDim.x >> 6) + int(threadIdx.x >> 6);
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
constexpr uint32_t kRowStack = kRowLeaf + kLeafShareWords;
constexpr uint32_t kRegenRowStack = kRegenLdsState;  // regenerating kernel: rows 0-8 as above, the stack from row 9

// Cost-ordered dispatch (HgKernelParams::tile_order): the wave's tile, read through the scalar cache (the order is
// written by hg_order_tiles before this launch and never during it).
__device__ __forceinline__ int ordered_tile(const HgKernelParams& kp, uint32_t w) {
    if (!kp.tile_order) return int(w);
    return int(kp.tile_order[w]);
}
// The wave's work unit (tile, frame chunk).  Tile-index order: chunk-major (wave w: tile w mod tiles, chunk
// w / tiles).  Cost order: tile-major (wave w: tile order[w / split], chunk w mod split), so a tile's chunks run side by
// side and the most expensive tiles' chunks all start first (tools/sweeps/sweep81.txt).  Waves past the last unit get
// chunk = split (no work).
__device__ __forceinline__ void wave_unit(const HgKernelParams& kp, uint32_t gw, uint32_t nlt, uint32_t split,
                                          int& tile, uint32_t& chunk) {
    if (kp.tile_order) {
        const uint32_t w = gw / split;
        tile = w < nlt ? ordered_tile(kp, w) : 0;
        chunk = w < nlt ? gw % split : split;
        return;
    }
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
    uint32_t nf;  // frames of the chunk
    __device__ TileItems() : tx0(0), ty0(0), tw(0), nv(0), n_items(0), f_begin(0), nf(1u) {}  // unused
    __device__ TileItems(const HgKernelParams& kp, int local_tile, bool valid, uint32_t fb, uint32_t fe, uint32_t lane) {
        const int g = __builtin_amdgcn_readfirstlane(kp.rank + local_tile * kp.n_ranks);
        tx0 = uint32_t(g % kp.tiles_x) * HG_TILE;
        ty0 = uint32_t(g / kp.tiles_x) * HG_TILE;
        tw = __builtin_amdgcn_readfirstlane(min(uint32_t(HG_TILE), kp.Wu - min(kp.Wu, tx0)));
        const uint32_t th = __builtin_amdgcn_readfirstlane(min(uint32_t(HG_TILE), kp.Hu - min(kp.Hu, ty0)));
        nv = tw * th;
        n_items = __builtin_amdgcn_readfirstlane(valid && fe > fb ? nv * (fe - fb) : 0u);
        f_begin = fb;
        nf = __builtin_amdgcn_readfirstlane(fe > fb ? fe - fb : 1u);
        if (lane == 0) hg_next_item = 64u;  // lane l starts with item l
        wave_lds_sync();
    }
    // item k -> valid pixel k / nf (its pixel within the tile, x + 8 y) and frame k mod nf: a wave's lanes trace one
    // pixel's frames (with the [slot][frame] colours: C3 +0.4 %, C2 +0.5 %, C5 -0.4 %; tools/sweeps/sweep_r02_be/bf)
    __device__ __forceinline__ void get(uint32_t k, uint32_t& pix, uint32_t& frame) const {
        uint32_t q, i;
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
// HG_CHECK_EXEC builds: words that every use leaves zeroed (the sort's histogram / claims / done count, a queue
// launch's heads and exit count) must read zero when the next use starts; each that does not counts into *faults
__global__ __launch_bounds__(64) void hg_check_zeroed(const uint32_t* __restrict__ p, uint32_t n,
                                                      unsigned long long* __restrict__ faults) {
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i < n && p[i] != 0u) atomicAdd(faults, 1ull);
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
#if HG_CHECK_EXEC
    if (faults)
        hipLaunchKernelGGL(hg_check_zeroed, dim3((2049u + 63u) / 64u), dim3(64), 0, stream,
                           static_cast<const uint32_t*>(scratch), 2049u, faults);
#endif
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
    const uint32_t gw = blockIdx.x;
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
            __builtin_amdgcn_s_setprio(HG_TRAVERSE_PRIO);
            const Hit hit = intersect<kMeshLds>(kp, ray, c, stk);
            __builtin_amdgcn_s_setprio(0);
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

// A word of uncached device memory read by a scalar load that bypasses the scalar cache (p uniform: a kernel argument).
// The blends read the context's lost word so (hg_server_gate: once a server frame was lost, every later blend into the
// accumulator is skipped until a clear or a checkpoint load resets the word), one load per workgroup.
__device__ __forceinline__ uint32_t sload_u32(const uint32_t* p) {  // (p uniform: a kernel argument)
    uint32_t v;
    asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}

// Frame-parallel epilogue: acc = acc*(1-w) + c_f*w for f in frame order (AccumulationShader.shader:33), exactly the
// per-frame blend the kernels do themselves when they blend in place.
// Over the [slot][frame] colour layout each wave owns 64 slots (a tile) and moves their colours 8 frames at
// a time through LDS, so every load instruction reads whole 128-B lines (8 lanes per line: one slot's 8 frames)
// instead of 64 lanes on 64 lines; then each lane blends its slot's 8 frames in frame order.
__global__ __launch_bounds__(256) void hg_blend_frames_sm(float4* __restrict__ acc, const float4* __restrict__ colors,
                                                          uint32_t n_slots, int32_t n_frames, int32_t first_frame,
                                                          int32_t accumulate, const uint32_t* lost) {
    if (sload_u32(lost)) return;
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

// The blend of a launch of few frames (at most HG_QUEUE_MAX_FRAMES): one thread per slot, no LDS, 64-thread groups and
// few registers.  A 1-frame launch's blend runs while the next launch's persistent trace waves hold the CUs' wave slots
// and most of their LDS: this one fits beside them (the LDS-staged hg_blend_frames_sm, 36 KB per group, waited for
// the trace to wind down: 0.7 ms per 1-frame blend on C3).  Same operations in the same order.
__global__ __launch_bounds__(64) void hg_blend_frames_lean(float4* __restrict__ acc, const float4* __restrict__ colors,
                                                           uint32_t n_slots, int32_t n_frames, int32_t first_frame,
                                                           int32_t accumulate, const uint32_t* lost) {
    if (sload_u32(lost)) return;
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= n_slots) return;
    float4 a = acc[i];
    for (int32_t f = 0; f < n_frames; ++f) {
        const float4 c = fc_load(colors + fc_slot_frame(i, uint32_t(f), uint32_t(n_frames)));
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

hipError_t hg_launch_blend_frames(const HgKernelParams& kp, const uint32_t* lost, hipStream_t stream) {
    const uint32_t n_slots = uint32_t(kp.n_local_tiles) * 64u;
    if (n_slots == 0) return hipSuccess;
    if (kp.n_frames <= HG_QUEUE_MAX_FRAMES) {
        hipLaunchKernelGGL(hg_blend_frames_lean, dim3((n_slots + 63) / 64), dim3(64), 0, stream, kp.acc, kp.frame_color,
                           n_slots, kp.n_frames, kp.first_frame, kp.accumulate, lost);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(hg_blend_frames_sm, dim3((n_slots + 255) / 256), dim3(256), 0, stream, kp.acc,
                       kp.frame_color, n_slots, kp.n_frames, kp.first_frame, kp.accumulate, lost);
    return hipGetLastError();
}

// LDS bytes with the mesh records after `base` bytes of rows, or 0 when they do not fit `budget` (or HG_MESH_LDS is off)
static size_t mesh_lds_bytes(size_t base, int32_t n_meshes, size_t budget) {
    if (n_meshes <= 0) return 0;
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
// (kQueue launches, not the server) a lane's take reached past the first unit (or found both spent): the loop top must
// refill.  Raised by the taking lanes, cleared by the refill; the loop top reads this one word instead of running the
// refill (lane 0's reads of the item count, the current unit and its end) on every trace / shade round.
__shared__ uint32_t hg_q_need;

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
    if (k >= a_end) lds_put(hg_q_need, 1u);  // the first unit is spent (the server's loop top refills every round)
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

// ---------------------------------------------------------------------------------------------------------------
// The render server (kServer): the persistent queue waves outlive hg_render calls.  The reference dispatches once per
// frame (RP:327, RP:406); a launch per frame ends with every wave draining its last paths, its other lanes idle (0.63 ms
// of a C3 frame's 1.2 ms).  Here one launch serves every frame the host posts while it lives:
// unit u of the server is (frame k = u / tiles, the tile at cost-order position u mod tiles), handed out through the
// same 8 per-XCD heads, bounded by the frames posted so far; so the lanes that frame k's last paths leave idle take
// frame k+1's items at once.  Which wave traces an item changes nothing: every item runs with the inputs the
// reference's dispatch of frame k gives its pixel (FrameCount = first_frame + k) and writes its own colour slot.
//   posting   the host raises the post word (pinned host memory: frames posted | stop << 32).  A wave that finds no
//             posted unit reads the device mirror of that word; at most one wave per HG_SV_POLL_TICKS reads the host
//             word itself (a ticket) and raises the mirror by atomic max.
//   frames    a wave counts, per frame in a window of 4 (LDS), the units it pulled and the items of them its lanes
//             finished; once they match, after a store drain, it adds the units to the frame's ring-slot count
//             (frames_done).  Colours go to the frame's ring slot, and the ring and the counts are uncached device
//             memory (no XCD's L2 holds their lines): the gate kernel on the context stream waits for the count, and
//             the blend after it reads the colours, whichever XCD wrote them (plain stores then the drain, then the
//             count's atomic: the colours are in memory before the count says so).
//   leaving   a wave with no item and no posted unit left waits (s_sleep); it leaves once the stop flag is in its view
//             and nothing posted is left to claim.  The stop flag comes from the host (server_stop), or from the close
//             handshake: after sv_idle_ticks with nothing new posted, one wave closes the server (sv_close).  It raises
//             the closing word in host memory, then reads the post word, and publishes what it read with the stop flag
//             (to the host and to every mirror): every frame it read is traced before the waves leave.  The host raises
//             the post word, then reads the closing word; a post that finds it raised counts only if the closing wave
//             read it (both sides store, then load: at least one sees the other's store), else the host restarts the
//             server and posts there.  So no posted frame can meet a server whose waves have all left.
// Only the lane 0 of a wave runs these (the whole wave converged at the loop top).
// Per-wave LDS state (lane 0 reads and writes it; the constants are copied from the kernel arguments once, so that no
// server value stays in a scalar register across the kernel's loop: its scalar registers are all taken, and every
// value kept live there spilled the traversal's vector registers to scratch — 84 B per lane in the first form)
struct SvWave {
    uint32_t view;   // units posted as this wave last saw them
    uint32_t dry;    // the view at which this wave last found every head dry (HG_NONE: none)
    uint32_t pend;   // a unit claimed beyond the view, or whose frame window was busy (HG_NONE: none)
    uint32_t more, more_n;  // the rest of a multi-unit claim: more_n units from `more` in steps of 8, after pend
    uint32_t stop;   // the stop flag as this wave last saw it
    uint32_t nlt, mask, cap, magic, shift, idle_ticks;  // tiles per frame, ring slots - 1, frames cap, u / nlt, leave after
    uint32_t post_lo, post_hi, done_lo, done_hi;        // the host post word and the ring-slot counts (pointers)
    uint32_t win_frame[4], win_units[4], win_items[4], win_done[4];  // frame window (k & 3)
};
__shared__ SvWave hg_sv;

__device__ __forceinline__ unsigned long long* sv_word64(const HgKernelParams& kp, uint32_t word) {
    return reinterpret_cast<unsigned long long*>(kp.queue + word);
}
// A control word read by a scalar load that bypasses the scalar cache (glc), from uncached memory (the runtime allocates
// the control block so: no L2 holds it either).  The polling of idle waves stays off the CU's vector-memory pipe, whose
// texture units return data in order: a vector poll of a contended coherent word held up the loads of the busy waves
// beside it (with the idle waves of a frame's end polling, a posted frame took several times its trace time).
__device__ __forceinline__ unsigned long long sv_sload(const unsigned long long* p) {
    unsigned long long v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}
// The same for a 32-bit word (a unit head); the address made wave-uniform (lane 0's branch: a value read from LDS
// counts as divergent).  readfirstlane returns int: each half through uint32_t, or a low half >= 2^31 would
// sign-extend over the high one.
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(a >> 32)));
    const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(a)));
    const uint32_t* const q = reinterpret_cast<const uint32_t*>((uint64_t(hi) << 32) | lo);
    uint32_t v;
    asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(q) : "memory");
    return v;
}
template <class T>
__device__ __forceinline__ T* sv_ptr(uint32_t lo, uint32_t hi) {
    return reinterpret_cast<T*>((uint64_t(hi) << 32) | lo);
}
__device__ void sv_init(const HgKernelParams& kp) {  // lane 0, at the kernel's start
    lds_put(hg_sv.view, 0u);
    lds_put(hg_sv.dry, HG_NONE);
    lds_put(hg_sv.pend, HG_NONE);
    lds_put(hg_sv.more_n, 0u);
    lds_put(hg_sv.stop, 0u);
    lds_put(hg_sv.nlt, uint32_t(kp.n_local_tiles));
    lds_put(hg_sv.mask, kp.sv_ring - 1u);
    lds_put(hg_sv.cap, kp.sv_frames_cap);
    lds_put(hg_sv.magic, kp.sv_div_magic);
    lds_put(hg_sv.shift, kp.sv_div_shift);
    lds_put(hg_sv.idle_ticks, kp.sv_idle_ticks);
    lds_put(hg_sv.post_lo, uint32_t(uintptr_t(kp.sv_post)));
    lds_put(hg_sv.post_hi, uint32_t(uintptr_t(kp.sv_post) >> 32));
    lds_put(hg_sv.done_lo, uint32_t(uintptr_t(kp.frames_done)));
    lds_put(hg_sv.done_hi, uint32_t(uintptr_t(kp.frames_done) >> 32));
    for (uint32_t w = 0; w < 4u; ++w) {
        lds_put(hg_sv.win_frame[w], 0u);
        lds_put(hg_sv.win_units[w], 0u);
        lds_put(hg_sv.win_items[w], 0u);
        lds_put(hg_sv.win_done[w], 0u);
    }
}
// frame of unit u: u / nlt by the host's multiplier (exact for every u < 2^31; a power of two nlt: magic 0, a shift)
__device__ __forceinline__ uint32_t sv_frame(uint32_t u) {
    const uint32_t m = lds_get(hg_sv.magic);
    return (m ? __umulhi(u, m) : u) >> lds_get(hg_sv.shift);
}
// the posted units of a post word value
__device__ __forceinline__ uint32_t sv_units(unsigned long long w) {
    const uint32_t cap = lds_get(hg_sv.cap);
    return (uint32_t(w) < cap ? uint32_t(w) : cap) * lds_get(hg_sv.nlt);
}
// Refresh the view from the device mirror of the post word
__device__ uint32_t sv_view(const HgKernelParams& kp) {
    uint32_t v = lds_get(hg_sv.view);
    const unsigned long long m = sv_sload(sv_word64(kp, HG_SV_MIRROR_WORD + 32u * (blockIdx.x % HG_SV_MIRRORS)));
    const uint32_t u = sv_units(m);
    // a post word with the stop flag is final: its count may be below the frames posted ahead of the host's calls
    // (hg_runtime.hip server_speculate), which are abandoned (the units already pulled are traced)
    if (u > v || ((m & HG_SV_STOP) && u != v)) {
        v = u;
        lds_put(hg_sv.view, v);
    }
    if (m & HG_SV_STOP) lds_put(hg_sv.stop, 1u);
    return v;
}
// Take this XCD's host-poll ticket if it is free, read the host word over PCIe (system scope) and raise every mirror
// copy; then refresh the view.  (Idle waves call it every few spins, busy ones when they find the heads dry.)
__device__ uint32_t sv_poll(const HgKernelParams& kp) {
    unsigned long long* const ticket = sv_word64(kp, HG_SV_TICKET_WORD + 32u * (blockIdx.x & 7u));
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    unsigned long long t = sv_sload(ticket);
    if (now >= t && __hip_atomic_compare_exchange_strong(ticket, &t, now + HG_SV_POLL_TICKS, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        const unsigned long long h = __hip_atomic_load(
            sv_ptr<const unsigned long long>(lds_get(hg_sv.post_lo), lds_get(hg_sv.post_hi)), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_SYSTEM);
        for (uint32_t m = 0; m < HG_SV_MIRRORS; ++m)
            __hip_atomic_fetch_max(sv_word64(kp, HG_SV_MIRROR_WORD + 32u * m), h, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
    return sv_view(kp);
}
// Pull the next posted unit into hg_qu[slot], its items numbered from `base` (empty when there is none for now)
__device__ void sv_pull(const HgKernelParams& kp, uint32_t slot, uint32_t base) {
    QueueUnit& q = hg_qu[slot];
    lds_put(q.base, base);
    lds_put(q.end, base);
    uint32_t u = lds_get(hg_sv.pend);
    uint32_t view = lds_get(hg_sv.view);
    if (u == HG_NONE) {
        if (view == lds_get(hg_sv.dry)) {  // every head was dry at this view: anything new posted?  (A busy wave
            view = sv_poll(kp);            // polls the host word too: no wave may be waiting to do it)
            if (view == lds_get(hg_sv.dry)) return;
        }
        const uint32_t x = blockIdx.x & 7u;
        uint32_t take = 1u;
        for (uint32_t t = 0; t < 8u && u == HG_NONE; ++t) {  // own XCD's head first, then steal
            const uint32_t h = (x + t) & 7u;
            const uint32_t n = ld_agent(kp.queue + 32u * h);
            if (h + 8u * n >= view) continue;
            // HG_SV_CLAIM units per atomic while the head holds posted units for as many claims of every wave of its
            // XCD (one wave per block): no frame's end is left to a wave holding several
            if (HG_SV_CLAIM > 1u) take = h + 8u * (n + HG_SV_CLAIM * (1u + gridDim.x / 8u)) < view ? HG_SV_CLAIM : 1u;
            u = h + 8u * atomicAdd(kp.queue + 32u * h, take);
        }
        if (u == HG_NONE) {
            lds_put(hg_sv.dry, view);
            return;
        }
        lds_put(hg_sv.more, u + 8u);  // (placed after u)
        lds_put(hg_sv.more_n, take - 1u);
    }
    if (u >= view) view = sv_view(kp);
    const uint32_t k = sv_frame(u), w = k & 3u;
    if (u >= view || (lds_get(hg_sv.win_units[w]) != 0u && lds_get(hg_sv.win_frame[w]) != k)) {
        lds_put(hg_sv.pend, u);  // (claimed past the posted frames by a race, or its frame window still busy): later
        return;
    }
    const uint32_t more_n = lds_get(hg_sv.more_n);  // the next unit of a multi-unit claim, if any, is pulled next
    lds_put(hg_sv.pend, more_n ? lds_get(hg_sv.more) : HG_NONE);
    if (more_n) {
        lds_put(hg_sv.more, lds_get(hg_sv.more) + 8u);
        lds_put(hg_sv.more_n, more_n - 1u);
    }
    if (HG_SV_DIAG_TIMES && k < 256u)  // (analysis builds) the frame's first claim: max of the complement
        __hip_atomic_fetch_max(sv_word64(kp, HG_SV_DIAG_WORD + 4u * k), ~(unsigned long long)__builtin_amdgcn_s_memrealtime(),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t i = u - k * lds_get(hg_sv.nlt);  // the unit's place in its frame
    if (HG_SV_TILE_RUN > 1u && !kp.tile_order) {
        // runs: head h (u % 8, the XCD whose waves pull it first) takes runs h, h + 8, ... of HG_SV_TILE_RUN consecutive
        // tiles, so a wave's and a CU's consecutive units are neighbours (the tail past the last whole round in place)
        constexpr uint32_t B = HG_SV_TILE_RUN;
        if (i < (lds_get(hg_sv.nlt) / (8u * B)) * (8u * B)) {
            const uint32_t h = i & 7u, n = i >> 3;
            i = (n / B) * (8u * B) + h * B + n % B;
        }
    }
    const int tile = ordered_tile(kp, i);
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
    lds_put(q.f_begin, k);
    lds_put(q.nf, 1u);
    lds_put(q.end, base + tw * th);
    lds_put(hg_sv.win_frame[w], k);
    lds_put(hg_sv.win_units[w], lds_get(hg_sv.win_units[w]) + 1u);
    lds_put(hg_sv.win_items[w], lds_get(hg_sv.win_items[w]) + tw * th);
}
// Frames of the window whose pulled items the lanes have all finished: after a drain of the wave's colour stores, their
// units go to the frame's ring-slot count
__device__ void sv_flush(const HgKernelParams& kp) {
    (void)kp;
    bool drained = false;
    for (uint32_t w = 0; w < 4u; ++w) {
        const uint32_t n = lds_get(hg_sv.win_units[w]);
        if (n == 0u || lds_get(hg_sv.win_done[w]) != lds_get(hg_sv.win_items[w])) continue;
        if (!drained) {  // every lane's colour stores complete before the count moves
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            __builtin_amdgcn_s_waitcnt(0);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            drained = true;
        }
        uint32_t* const done = sv_ptr<uint32_t>(lds_get(hg_sv.done_lo), lds_get(hg_sv.done_hi));
        __hip_atomic_fetch_add(done + 32u * (lds_get(hg_sv.win_frame[w]) & lds_get(hg_sv.mask)), n, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (HG_SV_DIAG_TIMES && lds_get(hg_sv.win_frame[w]) < 256u)  // (analysis builds) the frame's last count
            __hip_atomic_fetch_max(sv_word64(kp, HG_SV_DIAG_WORD + 4u * lds_get(hg_sv.win_frame[w]) + 2u),
                                   (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        lds_put(hg_sv.win_units[w], 0u);
        lds_put(hg_sv.win_items[w], 0u);
        lds_put(hg_sv.win_done[w], 0u);
    }
}
// Loop top: flush finished frames, keep both units filled (the spent one refilled after the other; both spent: two
// new units, in turn).  Returns true when the wave has no item to hand out now.
__device__ bool sv_refill(const HgKernelParams& kp) {
    sv_flush(kp);
    const uint32_t cnt = lds_get(hg_next_item);
    uint32_t a = lds_get(hg_q_cur);
    if (cnt >= lds_get(hg_qu[a].end)) {  // the first unit is spent
        const uint32_t b_end = lds_get(hg_qu[a ^ 1u].end);
        const bool both = cnt >= b_end;
        if (!both) lds_put(hg_q_cur, a ^ 1u);  // the second one is in use: it comes first now
        for (uint32_t i = 0; i < (both ? 2u : 1u); ++i) {  // (one inlined pull: every copy costs the loop registers)
            const uint32_t slot = a ^ i;
            sv_pull(kp, slot, i ? lds_get(hg_qu[a].end) : both ? cnt : b_end);
        }
        if (!both) a ^= 1u;
    }
    return cnt >= lds_get(hg_qu[a ^ 1u].end) && cnt >= lds_get(hg_qu[a].end);
}
// The close handshake (lane 0 of an idle wave, after sv_idle_ticks with nothing new posted).  One wave wins the closing
// word of the control block; it raises the host's closing word, then reads the post word (system scope, sequentially
// consistent: the store is visible to the host before the load is performed), and publishes the post word it read with
// the stop flag, to the host (the close word, HG_SV_CLOSED) and to every mirror (atomic max: the stop flag outranks
// every post word without it, so a poller that read a later post word cannot raise a view past it).  Every wave then
// drains the frames of that view and leaves.  The host's side is hg_runtime.hip server_post.
__device__ void sv_close(const HgKernelParams& kp) {
    uint32_t* const word = kp.queue + HG_SV_CLOSE_WORD;
    if (ld_agent(word) != 0u || atomicCAS(word, 0u, 1u) != 0u) return;  // another wave closes it
    unsigned long long* const host = sv_ptr<unsigned long long>(lds_get(hg_sv.post_lo), lds_get(hg_sv.post_hi));
    __hip_atomic_store(host + HG_SV_HOST_CLOSING, 1ull, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    const unsigned long long p = __hip_atomic_load(host + HG_SV_HOST_POST, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long fin = (p & 0xFFFFFFFFull) | HG_SV_STOP;
    __hip_atomic_store(host + HG_SV_HOST_CLOSED, fin | HG_SV_CLOSED, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
    for (uint32_t m = 0; m < HG_SV_MIRRORS; ++m)
        __hip_atomic_fetch_max(sv_word64(kp, HG_SV_MIRROR_WORD + 32u * m), fin, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
}
// A wave with no path: poll (the host word through the ticket) and wait until a unit is posted (returns 0: refill) or
// it may leave (1): the stop flag in its view and nothing posted left to claim.  A wave that saw nothing new posted for
// sv_idle_ticks closes the server (sv_close); it never leaves on its own clock.
__device__ uint32_t sv_wait(const HgKernelParams& kp) {
    hg_wave_cost[threadIdx.x >> 6] = nullptr;  // the wait is no tile's cost
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t seen = HG_NONE;  // the view at which the heads were last read
    uint32_t idle_view = lds_get(hg_sv.view);  // the view at t0 (a new post restarts the idle clock)
    for (uint32_t spin = 0;; ++spin) {
        // one coherent load per spin (this wave's mirror copy); the host word through the ticket every few spins
        const uint32_t view = (spin % HG_SV_POLL_EVERY) == 0u ? sv_poll(kp) : sv_view(kp);
        // A wave holding a unit (claimed past the posted ones by a race with another claimer, or with its frame
        // window busy) claims nothing else until it is placed: it waits for that unit alone.  (No wave set can end
        // up all holding unposted units while posted ones remain: the last claimer's overshoot needs a concurrent
        // claimer, which then holds none.)
        const uint32_t pend = lds_get(hg_sv.pend);
        bool open = pend != HG_NONE && pend < view;
        if (pend == HG_NONE && view != seen) {  // the heads, only when the posted units changed
            seen = view;
            for (uint32_t h = 0; h < 8u && !open; ++h) open = h + 8u * ld_agent(kp.queue + 32u * h) < view;
        }
        if (open) {
            lds_put(hg_sv.dry, HG_NONE);
            return 0u;
        }
        if (lds_get(hg_sv.stop)) return 1u;  // the final post word: nothing posted is left to claim
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (view != idle_view) {
            idle_view = view;
            t0 = now;
        } else if (now - t0 > uint64_t(lds_get(hg_sv.idle_ticks))) {
            sv_close(kp);  // (then the stop flag reaches this wave's view through the mirrors)
        }
        // short sleeps between the first polls, then longer ones (s_sleep counts 64 clocks)
        if (spin < HG_SV_SPIN_SHORT) __builtin_amdgcn_s_sleep(HG_SV_SLEEP_SHORT);
        else __builtin_amdgcn_s_sleep(HG_SV_SLEEP_LONG);
    }
}
// (the colour stores of a server frame: fc_store into the uncached ring)

// Streaming variant (HG_KERNEL_MEGA_STREAM): the regenerating kernel with a resumable traversal.  Lanes advance
// their traversal one while-while round at a time; once at most HG_STREAM_TMIN lanes are still traversing (and
// some have finished), the finished lanes shade their hit and start their next ray while the stragglers keep
// their traversal state, so the wave's lanes stay busy instead of waiting for the slowest ray of every bounce.
// Every frame's colour goes to frame_color (item scheduling), blended in frame order by hg_blend_frames.  kQueue: the
// persistent work-queue form above (launches of few frames).
// kServer (with kQueue): the render server's persistent form above.
template <bool kCounters, bool kMeshLds, bool kQueue, bool kDeep, bool kServer>
__global__ __launch_bounds__(HG_STREAM_LB, HG_STREAM_WAVES) void hg_trace_stream_kernel(const HgKernelParams kp) {
    static_assert(!kServer || kQueue, "the render server is a queue launch");
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
            lds_put(hg_q_need, 1u);  // (both units empty: the first loop top pulls two)
            hg_wave_cost[threadIdx.x >> 6] = nullptr;
            if constexpr (kServer) sv_init(kp);
        }
    } else {
        // wave -> (tile, frame chunk), as in hg_trace_regen_kernel
        // one wave per workgroup (launched with 64 threads): wave = workgroup
        const uint32_t gw = blockIdx.x;
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
    __builtin_amdgcn_s_setprio(HG_TRAVERSE_PRIO);  // traversal waits on memory: its waves issue first
    for (;;) {  // (kServer: once per stretch of posted work; the others: once)
        if constexpr (kServer) {  // (no path in flight: the state starts afresh, so none of it is live across the wait)
            work = false;
            ray = Ray{mk(0, 0, 0), mk(0, 0, 1)};
            tv = Trav{};
            tv.mi = nm;
            smp = Sampler{0u, 0u, 0u};
            ms = MediumStack{0ull, 0};
            fs = bounce = slot = 0u;
            acc_rough = 0.0f;
        }
        for (;;) {
            // ---- kQueue: the wave refills a spent unit, and idle lanes (the wave's start; lanes whose take found both
            // units spent) become fresh: they take their item in the shading pass below
            if constexpr (kServer) {
                wave_lds_sync();
                if (lane == 0u) lds_put(hg_q_empty, sv_refill(kp) ? 1u : 0u);
                wave_lds_sync();
                if (!work && __builtin_amdgcn_readfirstlane(lds_get(hg_q_empty)) == 0u) {
                    work = true;
                    bounce = kFreshLane;
                    tv.mi = nm;
                }
            } else if (kQueue && !dry) {
                wave_lds_sync();
                if (__builtin_amdgcn_readfirstlane(lds_get(hg_q_need)) != 0u) {  // (an idle lane implies a take past it)
                    if (lane == 0u) {
                        lds_put(hg_q_need, 0u);
                        lds_put(hg_q_empty, queue_refill(kp, n_units, split) ? 1u : 0u);
                    }
                    wave_lds_sync();
                    dry = __builtin_amdgcn_readfirstlane(lds_get(hg_q_empty)) != 0u;
                }
                if (!work && !dry) {
                    work = true;
                    bounce = kFreshLane;
                    tv.mi = nm;
                }
            }
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
            __builtin_amdgcn_s_setprio(0);
            // ---- finished lanes: shade, then start their next ray (a ray with nothing to traverse shades again)
            // (rays that finish at once — everything culled — shade again in this loop while at least
            // HG_STREAM_RESHADE lanes need it, otherwise in the next shading phase)
            for (uint32_t it = 0;; ++it) {
                const uint32_t n_sh = wave_count(work && tv.mi >= nm);
                if (n_sh == 0u || (it > 0u && n_sh < kReshade)) break;
                if (work && tv.mi >= nm) {
                c.shade_rounds += wave_once();
                const bool fresh = kQueue && bounce == kFreshLane;  // no path yet: straight to the take below
                bool alive = false;
                f3 thr = s_thr.get(), col = s_col.get();
                if (!fresh) {
                const Hit hit = trav_hit<kMeshLds>(kp, ray, tv);
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
                        // this frame's colour, blended later in frame order (hg_blend_frames*; the server's gate + blend)
                        if constexpr (kServer) {
                            if (!fresh) {
                                const uint32_t k = smp.frame - uint32_t(kp.first_frame);  // the server's frame index
                                // (the ring is uncached memory: the gate and blend on another XCD read what this wrote)
                                fc_store(kp.frame_color + size_t(k & lds_get(hg_sv.mask)) * (lds_get(hg_sv.nlt) * 64u) + slot_i,
                                         make_float4(color.x, color.y, color.z, 1.0f));
                                atomicAdd(&hg_sv.win_done[k & 3u], 1u);  // (LDS) one more item of frame k finished
                            }
                        } else if (!fresh) {
                            fc_store(kp.frame_color + fc_index(kp, fs >> 16, slot_i), make_float4(color.x, color.y, color.z, 1.0f));
                        }
                        fs = (fs & 0xFFFF0000u) + 0x10000u;
                        if constexpr (kQueue) {
                            uint32_t f = 0, hx = 0, hy = 0;
                            if (queue_item(queue_take(), slot, f, hx, hy)) {  // the unit's next item: statics reset
                                next = true;
                                sum = mk(0, 0, 0);
                                fs = kServer ? 0u : f << 16;  // (the server's frame index is smp.frame - first_frame)
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
                if (alive) trav_begin<kMeshLds>(kp, ray, tv, c);
                }
            }
            __builtin_amdgcn_s_setprio(HG_TRAVERSE_PRIO);
            if (kCounters) cyc_shade += wave_clock();
        }
        if constexpr (!kServer) {
            break;
        } else {
            // no path in flight and no item to hand out: wait for the host's next frame (polling the host word), or
            // leave.  Outside the tracing loop, where no path state is live (its registers stay the tracing loop's).
            wave_lds_sync();
            if (lane == 0u) lds_put(hg_q_empty, sv_wait(kp));
            wave_lds_sync();
            if (__builtin_amdgcn_readfirstlane(lds_get(hg_q_empty)) != 0u) break;
        }
    }
    if constexpr (kQueue) record_tile_cost(lane);
    else items.record_cost(kp, lane);
    if constexpr (kServer) {  // waves out | grid << 32 (the gates: a frame still short once all left is lost)
        if (lane == 0u) {
            // after this wave's frame counts (its last sv_flush) have completed in memory
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            __builtin_amdgcn_s_waitcnt(0);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            __hip_atomic_store(kp.queue + HG_SV_EXIT_WORD + 1u, gridDim.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(kp.queue + HG_SV_EXIT_WORD, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if constexpr (kQueue && !kServer) {
        // The last wave out resets the queue heads for the next launch on this stream (no memset launch per queue
        // launch: a blit kernel waited for a CU that the other streams' persistent waves held).  A wave leaves only
        // once its pulls found the queue dry, and it pulls no more after that: every head atomic of the launch has
        // returned before the last wave's increment of the exit count.  Relaxed: an agent-scope acquire / release is
        // a write-back / invalidate of the XCD's whole L2 on gfx950, per wave leaving (strict C3 +1.3 %, a display
        // one frame behind +3.4 % without it; DESIGN.md section 10 lever 13); the next launch on this stream starts
        // after this one's end.
        if (lane == 0u) {
            const uint32_t out = __hip_atomic_fetch_add(kp.queue + HG_QUEUE_DONE_WORD, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            if (out == gridDim.x - 1u) {
                for (uint32_t h = 0; h < 8u; ++h)
                    __hip_atomic_store(kp.queue + 32u * h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

hipError_t hg_launch_mega_stream(const HgKernelParams& kp_in, int block, bool counters, hipStream_t stream, bool server) {
    (void)block;  // one wave per workgroup (the kernel's LDS rows assume it)
    int64_t grid = int64_t(kp_in.n_local_tiles) * kp_in.frame_split;
    const bool queue = kp_in.queue != nullptr;  // the runtime passes a queue for launches of few frames
    if (queue) grid = grid < int64_t(kp_in.resident_waves) ? grid : int64_t(kp_in.resident_waves);  // persistent waves
    else if (kp_in.wave_units > 1u && kp_in.frame_split == 1)  // wave_units tiles per wave (UnitItems)
        grid = (grid + kp_in.wave_units - 1) / kp_in.wave_units;
    if (grid == 0) return hipSuccess;
    const uint32_t lds_depth = kp_in.stack_depth < HG_STREAM_LDS_STACK ? kp_in.stack_depth : HG_STREAM_LDS_STACK;
    const size_t lds = size_t(kRowStack + lds_depth) * 64u * sizeof(uint32_t);
    HgKernelParams kp = kp_in;
    kp.mesh_lds_word = uint32_t(lds / 4u);
    const size_t mesh_lds = mesh_lds_bytes(lds, kp.n_meshes, HG_WAVE_LDS_BUDGET);
    const dim3 g{uint32_t(grid)}, b{64u};
    const size_t sh = mesh_lds ? mesh_lds : lds;
#if HG_CHECK_EXEC
    if (queue && !server && kp.counters)  // the last wave of the previous launch zeroed the heads and the exit count
        hipLaunchKernelGGL(hg_check_zeroed, dim3((HG_QUEUE_BYTES / 4u + 63u) / 64u), dim3(64), 0, stream,
                           static_cast<const uint32_t*>(kp.queue), uint32_t(HG_QUEUE_BYTES / 4u), kp.counters + 18);
#endif
    // deep BLAS (kp.stream_deep): the kDeep thresholds
#define HG_STREAM_LAUNCH_S(C, M, Q, S)                                                                                 \
    do {                                                                                                               \
        if (kp.stream_deep) hipLaunchKernelGGL((hg_trace_stream_kernel<C, M, Q, true, S>), g, b, sh, stream, kp);     \
        else hipLaunchKernelGGL((hg_trace_stream_kernel<C, M, Q, false, S>), g, b, sh, stream, kp);                   \
    } while (0)
#define HG_STREAM_LAUNCH(C, M, Q) HG_STREAM_LAUNCH_S(C, M, Q, false)
    if (server) {
        if (counters && mesh_lds) HG_STREAM_LAUNCH_S(true, true, true, true);
        else if (counters) HG_STREAM_LAUNCH_S(true, false, true, true);
        else if (mesh_lds) HG_STREAM_LAUNCH_S(false, true, true, true);
        else HG_STREAM_LAUNCH_S(false, false, true, true);
    } else if (queue) {
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
#undef HG_STREAM_LAUNCH_S
    return hipGetLastError();
}

// The render server's per-frame work on the context stream (hg_runtime.hip server_post): the gate waits until the
// frame's ring-slot count reaches `target` (one wave; agent-scope polls with a sleep).  It gives up when every wave of
// the server has left with the count still short (the frame can no longer complete), or after `timeout_ticks`: then
// the frame is lost, and the gate raises the context's lost word (device memory: every later blend into the
// accumulator is skipped, until a clear or a checkpoint load resets it) and the host's lost-frame word (HG_SV_LOST |
// the accumulator epoch of the frame: the host marks the accumulator invalid).  The blend reads the frame's colours from
// the uncached ring and blends them into the accumulator: acc*(1-w) + c*w, w = 1/FrameCount
// (AccumulationShader.shader:33), the same operations as every other blend.  Both fit beside the server's waves
// (64-thread groups, no LDS, few registers).
__global__ __launch_bounds__(64) void hg_server_gate(const uint32_t* __restrict__ done, uint32_t target,
                                                     uint64_t timeout_ticks, const unsigned long long* exitw,
                                                     uint32_t* lost, unsigned long long* __restrict__ err,
                                                     uint32_t epoch) {
    // (the whole wave polls with scalar loads of uncached words: nothing on the vector-memory pipe of the CU it shares
    // with the server's waves; sv_sload)
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t spin = 0;; ++spin) {
        if (sload_u32(done) >= target) return;
        bool gone = false;
        if ((spin & 15u) == 15u) {  // every server wave has left: a count still short now stays short
            const unsigned long long w = sv_sload(exitw);
            gone = (w >> 32) != 0ull && uint32_t(w) == uint32_t(w >> 32) && sload_u32(done) < target;
        }
        if (gone || __builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) break;
        if (spin < 256u) __builtin_amdgcn_s_sleep(1);
        else __builtin_amdgcn_s_sleep(8);
    }
    if (threadIdx.x == 0) {
        __hip_atomic_store(lost, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(err, HG_SV_LOST | epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
__global__ __launch_bounds__(64) void hg_server_blend(float4* __restrict__ acc, const float4* __restrict__ colors,
                                                      uint32_t n_slots, int32_t frame_count, const uint32_t* lost) {
    if (sload_u32(lost)) return;  // a frame before this one was lost: the accumulator stays as it was
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= n_slots) return;
    const float4 c = fc_load(colors + i);  // (uncached memory: the server's stores, whichever XCD made them)
    float4 a = acc[i];
    const float w = rcp_exact(float(uint32_t(frame_count)));
    const float k = 1.0f - w;
    a = make_float4(a.x * k + c.x * w, a.y * k + c.y * w, a.z * k + c.z * w, a.w * k + 1.0f * w);
    acc[i] = a;
}
hipError_t hg_launch_server_frame(float4* acc, const float4* colors, uint32_t n_slots, int32_t frame_count,
                                  const uint32_t* done, uint32_t target, uint64_t timeout_ticks,
                                  const unsigned long long* exitw, uint32_t* lost, unsigned long long* err,
                                  uint32_t epoch, hipStream_t stream) {
    hipLaunchKernelGGL(hg_server_gate, dim3(1), dim3(64), 0, stream, done, target, timeout_ticks, exitw, lost, err,
                       epoch);
    if (n_slots)
        hipLaunchKernelGGL(hg_server_blend, dim3((n_slots + 63) / 64), dim3(64), 0, stream, acc, colors, n_slots,
                           frame_count, static_cast<const uint32_t*>(lost));
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
