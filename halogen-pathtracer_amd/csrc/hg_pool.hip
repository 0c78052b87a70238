// hg_pool.hip — path-pool megakernel (A/B variant HG_KERNEL_MEGA_POOL, built only with make VARIANTS=1:
// 1,160 Mpaths/s on C3).
//
// Same hot path as hg_trace_regen_kernel (HalgoenCompute.compute:1015-1063 + the accumulation blit), organised so
// that a wave's lanes stay busy during BVH traversal.  One wave owns HG_POOL_TILES 8x8 tiles (kPoolSlots paths,
// more than its 64 lanes); each path lives in a 128-B slot of a per-wave global array.  The wave alternates:
//   trace (mesh-major): for each mesh in buffer order, every queued ray whose exact-cull bit is set for that mesh
//          is traversed through it — lanes take the rays of that mesh's list and refill as soon as one finishes.
//          All lanes walk the same BVH (similar depths, shared top levels in cache); per ray the meshes are still
//          visited in buffer order with best_t carried in the slot, exactly the reference's order (:386-450);
//   shade: lanes take the traced slots 64 at a time, resolve and shade the hit (one body of trace_ray's loop,
//          :898-945), regenerate finished paths (next sample / frame, blending a finished frame into the
//          accumulator), and start the slot's next ray (spheres + mesh cull, :357-376, :386).
// Only the queue lengths are live across phases, so the register budget stays the regen kernel's.  Per ray the
// arithmetic and visit order are unchanged, so the image and the work counters are bit-identical.
#include <hip/hip_runtime.h>

#include "hg_device.h"

using namespace hgd;

constexpr uint32_t kPoolSlots = HG_POOL_TILES * 64u;
constexpr uint32_t kSlotF4 = 8;  // float4 per slot (layout below)

// Slot layout (float4 index): 0 = origin, accRoughness | 1 = direction, frame<<16|sample | 2 = throughput,
// bounce word | 3 = radiance, Sobol dimension offset | 4 = sample sum, medium stack depth | 5 = medium stack
// (u64), live-mesh mask (u64) | 6 = best t, u, v, triangle|orientation | 7 = best mesh, sphere ref, sphere t.
static_assert(kPoolSlots <= 1024, "pool too large for the LDS queues");

// number of lanes below this one whose bit is set in m
__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
}

struct PoolPixel {
    uint32_t px, py, slot_i;  // image pixel and accumulator slot (local tile * 64 + pixel in tile)
    bool valid;
};

__device__ __forceinline__ PoolPixel pool_pixel(const HgKernelParams& kp, uint32_t group, uint32_t s) {
    PoolPixel q;
    const uint32_t t = group * HG_POOL_TILES + (s >> 6), p = s & 63u;
    q.valid = t < uint32_t(kp.n_local_tiles);
    const int gtile = kp.rank + int(t) * kp.n_ranks;
    q.px = uint32_t(gtile % kp.tiles_x) * HG_TILE + (p & 7u);
    q.py = uint32_t(gtile / kp.tiles_x) * HG_TILE + (p >> 3);
    q.valid = q.valid && q.px < kp.Wu && q.py < kp.Hu;
    q.slot_i = t * 64u + p;
    return q;
}

// get_ray_intersection's per-ray prologue (:474-485, :357-381): sphere pass, exact mesh-cull mask; stores the
// ray and its running closest hit into the slot.
__device__ __forceinline__ void pool_begin_ray(const HgKernelParams& kp, float4* sl, const Ray& r, Counters& c,
                                               float4 s0w_acc_fs /* .x = accRoughness, .y = fs bits */) {
    c.rays++;
    float sph_t = HG_INF;
    const uint32_t sph = isect_spheres(kp, r, sph_t);
    uint32_t culled = 0;
    const f3 winv = mk(rcp_exact(r.d.x), rcp_exact(r.d.y), rcp_exact(r.d.z));
    const uint64_t live = mesh_live_mask(kp, r.o, winv, sph_t, culled);
    c.aabb += 2 * culled;
    sl[0] = make_float4(r.o.x, r.o.y, r.o.z, s0w_acc_fs.x);
    sl[1] = make_float4(r.d.x, r.d.y, r.d.z, s0w_acc_fs.y);
    sl[5].z = __uint_as_float(uint32_t(live));
    sl[5].w = __uint_as_float(uint32_t(live >> 32));
    sl[6] = make_float4(sph_t, 0.0f, 0.0f, __uint_as_float(HG_NONE));
    sl[7] = make_float4(__uint_as_float(0u), __uint_as_float(sph), sph_t, 0.0f);
}

template <bool kCounters>
__global__ __launch_bounds__(64, HG_POOL_WAVES) void hg_trace_pool_kernel(const HgKernelParams kp) {
    const uint32_t lane = threadIdx.x;
    const uint32_t gw = xcd_block(blockIdx.x, gridDim.x);
    const uint32_t nlt = uint32_t(kp.n_local_tiles), split = uint32_t(kp.frame_split);
    const uint32_t n_groups = (nlt + HG_POOL_TILES - 1) / HG_POOL_TILES;
    const uint32_t group = gw % n_groups, chunk = gw / n_groups;
    const uint32_t f_begin = uint32_t((uint64_t(chunk) * uint32_t(kp.n_frames)) / split);
    const uint32_t f_end = uint32_t((uint64_t(chunk + 1) * uint32_t(kp.n_frames)) / split);
    if (chunk >= split || f_end <= f_begin) return;  // wave-uniform

    const MegaStack stk{lane, 64u, kp.spill + blockIdx.x * 64u + lane, kp.spill_stride};
    const uint32_t lds_depth = kp.stack_depth < HG_MEGA_LDS_STACK ? kp.stack_depth : HG_MEGA_LDS_STACK;
    uint32_t* ready_q = hg_lds_stack + lds_depth * 64u;
    uint32_t* shade_q = ready_q + kPoolSlots;
    float4* pool = kp.pool + size_t(gw) * kPoolSlots * kSlotF4;
    const uint32_t nm = uint32_t(kp.n_meshes);
    Counters c{0, 0, 0, 0, 0, 0};
    uint32_t paths = 0;

    // ---- every pixel of the wave's tiles starts its first path of the chunk (HalogenCompute :1023-1033)
    uint32_t n_ready = 0;
    for (uint32_t k = 0; k < HG_POOL_TILES; ++k) {
        const uint32_t s = k * 64u + lane;
        const PoolPixel q = pool_pixel(kp, group, s);
        if (q.valid) {
            const uint32_t fs = f_begin << 16;
            const Sampler smp{kp.accumulate ? uint32_t(kp.first_frame) + f_begin : 1u, pcg_hash(q.px + q.py * kp.Wu),
                              0u};
            const Ray r = camera_ray(kp, smp, (float(q.px) / kp.W) * 2.0f - 1.0f, (float(q.py) / kp.H) * 2.0f - 1.0f);
            paths++;
            float4* sl = pool + s * kSlotF4;
            sl[2] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(0u));
            sl[3] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(0u));
            sl[4] = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(0));
            sl[5] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            pool_begin_ray(kp, sl, r, c, make_float4(0.0f, __uint_as_float(fs), 0.0f, 0.0f));
        }
        const uint64_t vm = __ballot(q.valid);
        if (q.valid) ready_q[n_ready + lane_rank(vm)] = s;
        n_ready += uint32_t(__popcll(vm));
    }
    __syncthreads();

    while (n_ready > 0) {
        // ---- trace phase, mesh-major: mesh by mesh, the queued rays whose cull bit is set walk its BVH
        for (uint32_t mi = 0; mi < nm; ++mi) {
            // the list of this mesh's rays (shade_q holds it during the trace phase)
            uint32_t n_list = 0;
            for (uint32_t b = 0; b < n_ready; b += 64u) {
                bool need = false;
                uint32_t s = 0;
                if (b + lane < n_ready) {
                    s = ready_q[b + lane];
                    if (mi >= 64u) {
                        need = true;
                    } else {
                        const float4 s5 = pool[s * kSlotF4 + 5];
                        const uint32_t w = mi < 32u ? __float_as_uint(s5.z) : __float_as_uint(s5.w);
                        need = (w >> (mi & 31u)) & 1u;
                    }
                }
                const uint64_t nm_ = __ballot(need);
                if (need) shade_q[n_list + lane_rank(nm_)] = s;
                n_list += uint32_t(__popcll(nm_));
            }
            if (n_list == 0) continue;
            __syncthreads();
            const float4* md4 = reinterpret_cast<const float4*>(kp.meshes + mi);  // wave-uniform: scalar loads
            const float4 c0 = md4[0], c1 = md4[1], c2 = md4[2], c3 = md4[3];
            const uint32_t root = __float_as_uint(md4[4].x);
            uint32_t head = 0;
            bool act = false;
            uint32_t cur = 0, node = HG_NONE, sp = 0, best_tri = HG_NONE, best_mesh = 0;
            float best_t = HG_INF, best_u = 0.0f, best_v = 0.0f;
            f3 lo = mk(0, 0, 0), ld = mk(0, 0, 0), inv = mk(0, 0, 0);
            for (;;) {
                const uint64_t idle = __ballot(!act);
                if (idle != 0 && head < n_list) {
                    if (!act) {
                        const uint32_t r = head + lane_rank(idle);
                        if (r < n_list) {
                            cur = shade_q[r];
                            const float4* sl = pool + cur * kSlotF4;
                            const float4 o = sl[0], d = sl[1], h6 = sl[6], h7 = sl[7];
                            best_t = h6.x;
                            best_u = h6.y;
                            best_v = h6.z;
                            best_tri = __float_as_uint(h6.w);
                            best_mesh = __float_as_uint(h7.x);
                            // world -> local, direction NOT normalized (:390-392)
                            lo = mk(((c0.x * o.x + c1.x * o.y) + c2.x * o.z) + c3.x * 1.0f,
                                    ((c0.y * o.x + c1.y * o.y) + c2.y * o.z) + c3.y * 1.0f,
                                    ((c0.z * o.x + c1.z * o.y) + c2.z * o.z) + c3.z * 1.0f);
                            ld = mk(((c0.x * d.x + c1.x * d.y) + c2.x * d.z) + c3.x * 0.0f,
                                    ((c0.y * d.x + c1.y * d.y) + c2.y * d.z) + c3.y * 0.0f,
                                    ((c0.z * d.x + c1.z * d.y) + c2.z * d.z) + c3.z * 0.0f);
                            inv = mk(rcp_exact(ld.x), rcp_exact(ld.y), rcp_exact(ld.z));
                            node = root;  // root pushed untested (:401)
                            sp = 0;
                            act = true;
                        }
                    }
                    const uint32_t took = uint32_t(__popcll(idle));
                    head = (n_list - head < took) ? n_list : head + took;
                }
                if (!__any(act)) break;
                for (;;) {  // relaxed while-while, as in isect_meshes
                    const uint32_t n_desc = uint32_t(__popcll(__ballot(act && !(node & HG_LEAF_BIT))));
                    if (n_desc == 0u) break;
                    if (n_desc <= kp.descent_t && n_desc != uint32_t(__popcll(__ballot(act)))) break;
                    c.node_rounds += wave_once();
                    if (act && !(node & HG_LEAF_BIT)) {
                        const NodePair np = node_pair(kp, node);
                        float dA, dB;
                        pair_dist(np, lo, inv, dA, dB);
                        c.aabb += 2;
                        const uint32_t refA = pair_ref_a(np), refB = pair_ref_b(np);
                        const bool bFirst = dB < dA;  // :430-444
                        const uint32_t nearRef = bFirst ? refB : refA, farRef = bFirst ? refA : refB;
                        const bool nearOk = (bFirst ? dB : dA) < best_t, farOk = (bFirst ? dA : dB) < best_t;
                        if (nearOk) {
                            if (farOk) stk.push(sp, farRef);
                            node = nearRef;
                        } else if (farOk) {
                            node = farRef;
                        } else {
                            node = sp > 0 ? stk.pop(sp) : HG_NONE;
                        }
                    }
                }
                if (act && node != HG_NONE && (node & HG_LEAF_BIT)) {  // leaf (:404-420)
                    const uint2 leaf = leaf_range(kp, node);
                    const uint32_t end = leaf.x + leaf.y;
                    for (uint32_t ti = leaf.x; ti < end; ++ti) {
                        c.tri_rounds += wave_once();
                        float4 a, b;
                        float cz;
                        tri_load(kp, ti, a, b, cz);
                        c.tri++;
                        float tt, U, V;
                        bool front;
                        if (tri_accept(lo, ld, a, b, cz, best_t, tt, U, V, front)) {
                            best_t = tt;
                            best_u = U;
                            best_v = V;
                            best_tri = ti | (front ? 0u : 0x80000000u);
                            best_mesh = mi;
                        }
                    }
                    node = sp > 0 ? stk.pop(sp) : HG_NONE;
                }
                if (act && node == HG_NONE) {  // this ray is done with this mesh: running best back to the slot
                    float4* sl = pool + cur * kSlotF4;
                    sl[6] = make_float4(best_t, best_u, best_v, __uint_as_float(best_tri));
                    sl[7].x = __uint_as_float(best_mesh);
                    act = false;
                }
            }
            __syncthreads();
        }
        const uint32_t n_shade = n_ready;
        for (uint32_t b = 0; b < n_shade; b += 64u)  // shade every traced ray: the ready queue is the shade list
            if (b + lane < n_shade) shade_q[b + lane] = ready_q[b + lane];
        __syncthreads();
        // ---- shade phase: 64 finished slots at a time
        n_ready = 0;
        for (uint32_t b = 0; b < n_shade; b += 64u) {
            bool queue = false;
            uint32_t s = 0;
            if (b + lane < n_shade) {
                s = shade_q[b + lane];
                float4* sl = pool + s * kSlotF4;
                const float4 s0 = sl[0], s1 = sl[1], s2 = sl[2], s3 = sl[3], s4 = sl[4], s5 = sl[5], s6 = sl[6],
                             s7 = sl[7];
                const PoolPixel q = pool_pixel(kp, group, s);
                Ray r{xyz(s0), xyz(s1)};
                float acc_rough = s0.w;
                uint32_t fs = __float_as_uint(s1.w), bounce = __float_as_uint(s2.w);
                f3 thr = xyz(s2), col = xyz(s3);
                MediumStack ms{uint64_t(__float_as_uint(s5.x)) | (uint64_t(__float_as_uint(s5.y)) << 32),
                               __float_as_int(s4.w)};
                Sampler smp{kp.accumulate ? uint32_t(kp.first_frame) + (fs >> 16) : 1u, pcg_hash(q.px + q.py * kp.Wu),
                            __float_as_uint(s3.w)};
                Trav th;
                th.best_t = s6.x;
                th.best_u = s6.y;
                th.best_v = s6.z;
                th.best_tri = __float_as_uint(s6.w);
                th.best_mesh = __float_as_uint(s7.x);
                th.sph = __float_as_uint(s7.y);
                th.sph_t = s7.z;
                const Hit hit = trav_hit(kp, r, th);
                bool alive = false;
                if (hit.t < kp.far_) {  // :898-936
                    c.hits++;
                    const Mat mt = load_mat(kp, hit.mat);
                    col = col + xyz(mt.emis_rough) * thr;
                    uint32_t bt = 0;
                    const f3 att = evaluate_hit(kp, smp, ms, r, hit, mt, bt);
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
                    col = col + sample_sky(kp, r.d, sky_level(kp, acc_rough)) * thr;
                }
                f3 sum = xyz(s4);
                if (!alive) {
                    sum = sum + col;  // RayColor += trace_ray(...)
                    ++fs;
                    bool next = (fs & 0xFFFFu) < kp.spp;  // next sample: statics persist (:188-189)
                    if (!next) {
                        const float sppf = float(kp.spp);
                        const f3 color = mk(sum.x / sppf, sum.y / sppf, sum.z / sppf);
                        if (split > 1u) {  // frame-parallel: this frame's colour, blended later in frame order
                            kp.frame_color[fc_index(kp, fs >> 16, q.slot_i)] =
                                make_float4(color.x, color.y, color.z, 1.0f);
                        } else {
                            float4* slot = kp.acc + q.slot_i;
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
                        if ((fs >> 16) < f_end) {  // next frame = next dispatch: statics reset
                            next = true;
                            sum = mk(0, 0, 0);
                            smp.frame = kp.accumulate ? uint32_t(kp.first_frame) + (fs >> 16) : 1u;
                            smp.offset = 0;
                            ms = MediumStack{0ull, 0};
                        }
                    }
                    if (next) {
                        r = camera_ray(kp, smp, (float(q.px) / kp.W) * 2.0f - 1.0f,
                                       (float(q.py) / kp.H) * 2.0f - 1.0f);
                        thr = mk(1, 1, 1);
                        col = mk(0, 0, 0);
                        acc_rough = 0.0f;
                        bounce = 0;
                        paths++;
                        alive = true;
                    }
                }
                if (alive) {
                    sl[2] = make_float4(thr.x, thr.y, thr.z, __uint_as_float(bounce));
                    sl[3] = make_float4(col.x, col.y, col.z, __uint_as_float(smp.offset));
                    sl[4] = make_float4(sum.x, sum.y, sum.z, __int_as_float(ms.sp));
                    sl[5] = make_float4(__uint_as_float(uint32_t(ms.s)), __uint_as_float(uint32_t(ms.s >> 32)), 0.0f,
                                        0.0f);
                    pool_begin_ray(kp, sl, r, c, make_float4(acc_rough, __uint_as_float(fs), 0.0f, 0.0f));
                    queue = true;
                }
            }
            const uint64_t qm = __ballot(queue);
            if (queue) ready_q[n_ready + lane_rank(qm)] = s;
            n_ready += uint32_t(__popcll(qm));
        }
        __syncthreads();
    }
    if (kCounters) {
        const uint32_t v[9] = {paths, c.rays, c.tri, c.aabb, c.rays * nm, c.rays * uint32_t(kp.n_spheres), c.hits,
                               c.node_rounds, c.tri_rounds};
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint32_t sv = wave_sum(v[k]);
            if (lane == 0 && sv) atomicAdd(kp.counters + k, (unsigned long long)sv);
        }
        const uint32_t pm = wave_sum(c.primary_miss);
        if (lane == 0 && pm) atomicAdd(kp.counters + 16, (unsigned long long)pm);
    }
}

uint32_t hg_pool_slots() { return kPoolSlots; }
uint32_t hg_pool_tiles() { return HG_POOL_TILES; }

size_t hg_pool_lds_bytes(uint32_t stack_depth) {
    const uint32_t d = stack_depth < HG_MEGA_LDS_STACK ? stack_depth : HG_MEGA_LDS_STACK;
    return (size_t(d) * 64u + 2u * kPoolSlots) * sizeof(uint32_t);
}

// grid = pool groups x frame split, one wave per workgroup
hipError_t hg_launch_mega_pool(const HgKernelParams& kp, bool counters, hipStream_t stream) {
    const uint32_t n_groups = (uint32_t(kp.n_local_tiles) + HG_POOL_TILES - 1) / HG_POOL_TILES;
    const uint32_t grid = n_groups * uint32_t(kp.frame_split);
    if (grid == 0) return hipSuccess;
    const size_t lds = hg_pool_lds_bytes(kp.stack_depth);
    if (counters)
        hipLaunchKernelGGL(hg_trace_pool_kernel<true>, dim3(grid), dim3(64), lds, stream, kp);
    else
        hipLaunchKernelGGL(hg_trace_pool_kernel<false>, dim3(grid), dim3(64), lds, stream, kp);
    return hipGetLastError();
}
