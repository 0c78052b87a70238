// hg_wavefront.hip — the regenerating wavefront pipeline (A/B variant HG_KERNEL_WAVEFRONT, built only with
// make VARIANTS=1: 441 Mpaths/s on C3 against 2,400 for the streaming megakernel).
//
// Same semantics as the reference kernel HalogenCompute (HalgoenCompute.compute:1015-1063) + the
// accumulation blit (AccumulationShader.shader:27-34), bit for bit, but scheduled for gfx950:
//
//   hg_wf_gen    once per hg_render: starts frame 0 / sample 0 of every pixel slot (camera ray, get_ray
//                :996-1013), appends the slots to queue 0.
//   hg_wf_trace  per bounce: a PERSISTENT kernel that pulls rays from the current queue with wave-aggregated
//                atomics and runs get_ray_intersection (:474-485): sphere loop, then every mesh's BLAS.  It
//                holds only ray + traversal state (LDS stack [depth][lane], current node in a register), so
//                it runs at high occupancy, and a lane whose ray is done refills from the queue instead of
//                idling while its wave-mates traverse.
//   hg_wf_shade  per bounce: one body of trace_ray's loop (:889-947) for every queued path — emission,
//                evaluate_material_hit (medium stack + material_BRDF), Russian roulette, sky on a miss — and
//                compaction of the surviving paths into the next queue (64-bit __ballot + one atomic per wave).
//                A finished path REGENERATES its slot in place: the next sample of the same frame (statics
//                persist, :188-189) or the next frame (FrameCount+1, statics reset), after blending the
//                frame into the accumulation buffer (acc*(1-1/N) + new*(1/N)).  Pixels with short paths thus
//                keep feeding the queue until all their frames are done: no per-bounce SIMD idling and no
//                per-frame tail.
//
// Traversal order inside a BLAS is exactly the reference's (pop; leaf -> triangles in order; inner -> push
// far then near when tEntry < closest), so ties and pruning resolve identically; only the scheduling of
// independent rays differs.
#include <hip/hip_runtime.h>

#include "hg_device.h"

using namespace hgd;

namespace {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Append `slot` to queue when `alive` (all 64 lanes must call).  One atomic per wave.
__device__ __forceinline__ void wave_append(bool alive, uint32_t slot, uint32_t* __restrict__ queue,
                                            uint32_t* __restrict__ count) {
    const uint64_t m = __ballot(alive);
    if (m == 0) return;
    const uint32_t lane = lane_id();
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (int(lane) == leader) base = atomicAdd(count, uint32_t(__popcll(m)));
    base = __shfl(base, leader, 64);
    if (alive) queue[base + uint32_t(__popcll(m & ((1ull << lane) - 1ull)))] = slot;
}

__device__ __forceinline__ void slot_pixel(const HgKernelParams& kp, uint32_t slot, uint32_t& px, uint32_t& py) {
    const uint32_t lt = slot >> 6, lane = slot & 63u;
    const uint32_t gt = uint32_t(kp.rank) + lt * uint32_t(kp.n_ranks);
    px = (gt % uint32_t(kp.tiles_x)) * HG_TILE + (lane & 7u);
    py = (gt / uint32_t(kp.tiles_x)) * HG_TILE + (lane >> 3);
}

__device__ __forceinline__ Ray camera_ray_for(const HgKernelParams& kp, uint32_t px, uint32_t py, uint32_t frame,
                                              uint32_t offset) {
    const float ndcx = (float(px) / kp.W) * 2.0f - 1.0f;  // :1023-1024
    const float ndcy = (float(py) / kp.H) * 2.0f - 1.0f;
    const Sampler smp{frame, pcg_hash(px + py * kp.Wu), offset};
    return camera_ray(kp, smp, ndcx, ndcy);
}

__device__ __forceinline__ uint32_t frame_count(const HgKernelParams& kp, uint32_t f) {
    return kp.accumulate ? uint32_t(kp.first_frame) + f : 1u;
}

__device__ __forceinline__ void wave_add_counters(const HgKernelParams& kp, const uint32_t (&v)[7]) {
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const uint32_t s = wave_sum(v[k]);
        if (lane_id() == 0 && s) atomicAdd(kp.counters + k, (unsigned long long)s);
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------------------------
// gen: frame 0, sample 0 of every valid slot
// ---------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void hg_wf_gen(const HgKernelParams kp, uint32_t* __restrict__ q_out,
                                                 uint32_t* __restrict__ n_out) {
    uint32_t paths = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t base = blockIdx.x * blockDim.x; base < kp.n_slots; base += stride) {
        const uint32_t slot = base + threadIdx.x;
        bool alive = false;
        if (slot < kp.n_slots) {
            uint32_t px, py;
            slot_pixel(kp, slot, px, py);
            if (px < kp.Wu && py < kp.Hu) {
                alive = true;
                const Ray r = camera_ray_for(kp, px, py, frame_count(kp, 0), 0u);
                kp.p_o[slot] = make_float4(r.o.x, r.o.y, r.o.z, 0.0f);
                kp.p_d[slot] = make_float4(r.d.x, r.d.y, r.d.z, 0.0f);
                kp.p_thr[slot] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
                kp.p_col[slot] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                kp.p_sum[slot] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                kp.p_st[slot] = make_uint4(0, 0, 0, 0);
                kp.p_st2[slot] = make_uint4(0, 0, 0, 0);
                kp.p_ms[slot] = make_uint2(0, 0);
                paths++;
            }
        }
        wave_append(alive, slot, q_out, n_out);
    }
    if (kp.counters) {
        const uint32_t v[7] = {paths, 0, 0, 0, 0, 0, 0};
        wave_add_counters(kp, v);
    }
}

// ---------------------------------------------------------------------------------------------------------
// trace: persistent BLAS traversal over the queue
// ---------------------------------------------------------------------------------------------------------
namespace {
enum : uint32_t { ST_IDLE = 0, ST_MESH = 1, ST_TRAV = 2 };

using WfStack = Stack<HG_LDS_STACK>;

// first mesh index >= m that is not culled (meshes beyond 64 carry no cull bit and are always visited)
__device__ __forceinline__ uint32_t next_live(uint64_t live, uint32_t m) {
    if (m >= 64u) return m;
    const uint64_t b = live & (~0ull << m);
    return b ? uint32_t(__builtin_ctzll(b)) : 64u;
}

}  // namespace

template <bool kCounters>
__global__ __launch_bounds__(256, HG_TRACE_WAVES) void hg_wf_trace(const HgKernelParams kp, const uint32_t* __restrict__ q_in,
                                                   const uint32_t* __restrict__ n_in, uint32_t* __restrict__ head) {
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    const WfStack stk{threadIdx.x, blockDim.x, kp.spill + gtid, kp.spill_stride};
    const uint32_t n = *n_in;
    const float eps = 0.0001f;

    uint32_t c_rays = 0, c_tri = 0, c_aabb = 0;
    uint32_t st = ST_IDLE;
    bool exhausted = false;
    uint32_t slot = 0, mi = 0, node = HG_NONE, sp = 0;
    f3 lo = mk(0, 0, 0), ld = mk(0, 0, 0), inv = mk(0, 0, 0);
    float best_t = HG_INF, best_u = 0.0f, best_v = 0.0f, sph_t = HG_INF;
    uint32_t best_tri = HG_NONE, best_mesh = 0, sph_io = HG_NONE;  // sph_io: sphere index | orientation<0 << 31
    uint64_t live = ~0ull;  // meshes < 64 not skipped by the exact cull (meshes >= 64 are always traversed)

    for (;;) {
        // ---- refill idle lanes (wave-aggregated dequeue) ----
        {
            const bool want = st == ST_IDLE && !exhausted;
            const uint64_t m = __ballot(want);
            // batch dequeues: one atomic per >= refill_min rays keeps the shared head word far from saturation
            if (m && (uint32_t(__popcll(m)) >= kp.refill_min || !__any(st != ST_IDLE))) {
                const uint32_t lane = lane_id();
                const int leader = __ffsll((unsigned long long)m) - 1;
                uint32_t base = 0;
                if (int(lane) == leader) base = atomicAdd(head, uint32_t(__popcll(m)));
                base = __shfl(base, leader, 64);
                if (want) {
                    const uint32_t idx = base + uint32_t(__popcll(m & ((1ull << lane) - 1ull)));
                    if (idx < n) {
                        slot = q_in[idx];
                        const float4 o4 = kp.p_o[slot], d4 = kp.p_d[slot];
                        const f3 wo = mk(o4.x, o4.y, o4.z), wd = mk(d4.x, d4.y, d4.z);
                        c_rays++;
                        // get_ray_scene_intersection_sphere :357-376
                        const f3 winv = mk(rcp_exact(wd.x), rcp_exact(wd.y), rcp_exact(wd.z));
                        sph_t = HG_INF;
                        sph_io = HG_NONE;
                        for (int i = 0; i < kp.n_spheres; ++i) {
                            const float4 cr = kp.spheres[3 * i];
                            const float4 am = kp.spheres[3 * i + 1];
                            const float4 bb = kp.spheres[3 * i + 2];
                            if (!(ray_aabb(xyz(am), xyz(bb), wo, winv) < kp.far_)) continue;
                            const f3 sh = wo - xyz(cr);
                            const float bq = 2.0f * dot(sh, wd);
                            const float cq = dot(sh, sh) - cr.w * cr.w;
                            const float disc = bq * bq - 4.0f * cq;
                            if (!(disc >= 0.0f)) continue;
                            float hd = (-bq - __builtin_sqrtf(disc)) / 2.0f;
                            uint32_t back = 0;
                            if (hd < 0.0f) {
                                hd = (-bq + __builtin_sqrtf(disc)) / 2.0f;
                                back = 0x80000000u;
                            }
                            if (hd < sph_t && hd > eps) {
                                sph_t = hd;
                                sph_io = uint32_t(i) | back;
                            }
                        }
                        best_t = sph_t;  // closestIntersection.rayT = closestHit.rayT (:381)
                        best_tri = HG_NONE;
                        // Exact mesh skip (see HgDevMesh::cull_*): a mesh whose root children the ray certainly
                        // misses, or meets only beyond best_t, is not traversed; its 2 AABB tests are counted.
                        // best_t only decreases afterwards, so the verdict stays valid for the whole ray.
                        live = ~0ull;
                        const float lim = best_t * 1.0001f + 1e-4f;
                        const int ncull = kp.n_meshes < 64 ? kp.n_meshes : 64;
                        for (int m = 0; m < ncull; ++m) {
                            const HgDevMesh& md = kp.meshes[m];
                            if (!md.cullable) continue;
                            const float dA = ray_aabb(xyz(md.cull_a_lo), xyz(md.cull_a_hi), wo, winv);
                            const float dB = ray_aabb(xyz(md.cull_b_lo), xyz(md.cull_b_hi), wo, winv);
                            // a miss returns +INF (skip even when lim is INF); NaN never skips
                            const bool farA = dA == HG_INF || dA > lim, farB = dB == HG_INF || dB > lim;
                            if (farA && farB) {
                                live &= ~(1ull << m);
                                c_aabb += 2;
                            }
                        }
                        mi = next_live(live, 0);
                        st = ST_MESH;
                    } else {
                        exhausted = true;
                    }
                }
            }
            if (!__any(st != ST_IDLE)) break;
        }

        // ---- mesh setup / ray finish ----
        if (st == ST_MESH) {
            if (mi < uint32_t(kp.n_meshes)) {
                const float4* md = reinterpret_cast<const float4*>(kp.meshes + mi);
                const float4 c0 = md[0], c1 = md[1], c2 = md[2], c3 = md[3];  // worldToLocal columns
                const uint32_t root = __float_as_uint(md[4].x);
                const float4 o4 = kp.p_o[slot], d4 = kp.p_d[slot];  // world ray (L1/L2-resident)
                // mul(worldToLocal, float4(o,1)) / float4(d,0), direction NOT normalized (:390-392)
                lo = mk(((c0.x * o4.x + c1.x * o4.y) + c2.x * o4.z) + c3.x * 1.0f,
                        ((c0.y * o4.x + c1.y * o4.y) + c2.y * o4.z) + c3.y * 1.0f,
                        ((c0.z * o4.x + c1.z * o4.y) + c2.z * o4.z) + c3.z * 1.0f);
                ld = mk(((c0.x * d4.x + c1.x * d4.y) + c2.x * d4.z) + c3.x * 0.0f,
                        ((c0.y * d4.x + c1.y * d4.y) + c2.y * d4.z) + c3.y * 0.0f,
                        ((c0.z * d4.x + c1.z * d4.y) + c2.z * d4.z) + c3.z * 0.0f);
                inv = mk(rcp_exact(ld.x), rcp_exact(ld.y), rcp_exact(ld.z));
                node = root;  // root pushed untested (:401), held in a register
                sp = 0;
                st = ST_TRAV;
            } else {
                // :452 final accept; hit record for the shade kernel
                float4 tuvo;
                uint2 id;
                if (best_t < (sph_t - eps) && best_t < kp.far_) {
                    tuvo = make_float4(best_t, best_u, best_v, __uint_as_float(0x3F800000u | (best_tri & 0x80000000u)));
                    id = make_uint2(best_tri & 0x7FFFFFFFu, best_mesh);
                } else if (sph_io != HG_NONE) {
                    tuvo = make_float4(sph_t, 0.0f, 0.0f, (sph_io & 0x80000000u) ? -1.0f : 1.0f);
                    id = make_uint2((sph_io & 0x7FFFFFFFu) | HG_SPHERE_BIT, 0u);
                } else {
                    tuvo = make_float4(HG_INF, 0.0f, 0.0f, 0.0f);
                    id = make_uint2(HG_NONE, 0u);
                }
                kp.h_tuvo[slot] = tuvo;
                kp.h_id[slot] = id;
                st = ST_IDLE;
            }
        }

        // ---- inner nodes (while-while: all lanes descend together until each holds a leaf) ----
        while (__any(st == ST_TRAV && !(node & HG_LEAF_BIT))) {
            if (st == ST_TRAV && !(node & HG_LEAF_BIT)) {
                const NodePair np = node_pair(kp, node);
                float dA, dB;
                pair_dist(np, lo, inv, dA, dB);
                c_aabb += 2;
                const uint32_t refA = pair_ref_a(np), refB = pair_ref_b(np);
                // reference: push far, push near, pop near (:430-444) == keep near in the register
                const bool bFirst = dB < dA;
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

        // ---- one leaf per lane: triangles tested branch-free, the next one's loads issued ahead ----
        if (st == ST_TRAV && node != HG_NONE) {
            const uint2 leaf = leaf_range(kp, node);
            uint32_t ti = leaf.x;
            const uint32_t end = leaf.x + leaf.y;
            float4 ta, tb;
            float tc;
            tri_load(kp, ti, ta, tb, tc);
            for (; ti < end; ++ti) {
                const float4 a = ta, b = tb;
                const float cz = tc;
                if (ti + 1 < end) {
                    tri_load(kp, ti + 1, ta, tb, tc);
                }
                c_tri++;
                // triangle_intersection_doublesided :307-355 (all terms computed, one combined accept)
                const f3 e1 = mk(a.w, b.x, b.y);
                const f3 e2 = mk(b.z, b.w, cz);
                const f3 pvec = cross(ld, e2);
                const float det = dot(pvec, e1);
                const float inv_det = rcp_exact(det);
                const f3 tvec = lo - xyz(a);
                const float U = dot(tvec, pvec) * inv_det;
                const f3 qvec = cross(tvec, e1);
                const float V = dot(ld, qvec) * inv_det;
                const float t = dot(e2, qvec) * inv_det;
                const bool ok = !(fabsf(det) < 0.00000001f) && !(U < 0.0f || U > 1.0f) && !(V < 0.0f || U + V > 1.0f) &&
                                t > 0.0f && t > eps && t < best_t;
                if (ok) {
                    best_t = t;
                    best_u = U;
                    best_v = V;
                    best_tri = ti | (det > 0.0f ? 0u : 0x80000000u);  // orientation = sign(det)
                    best_mesh = mi;
                }
            }
            node = sp > 0 ? stk.pop(sp) : HG_NONE;
        }
        if (st == ST_TRAV && node == HG_NONE) {
            mi = next_live(live, mi + 1);
            st = ST_MESH;
        }
    }
    if (kCounters) {
        // every ray visits every mesh and tests every sphere prefilter: those counts follow from c_rays
        const uint32_t v[7] = {0, c_rays, c_tri, c_aabb, c_rays * uint32_t(kp.n_meshes),
                               c_rays * uint32_t(kp.n_spheres), 0};
        wave_add_counters(kp, v);
    }
}

// ---------------------------------------------------------------------------------------------------------
// shade: one loop body of trace_ray per queued path, then compaction / regeneration
// ---------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void hg_wf_shade(const HgKernelParams kp, const uint32_t* __restrict__ q_in,
                                                   const uint32_t* __restrict__ n_in, uint32_t* __restrict__ q_out,
                                                   uint32_t* __restrict__ n_out) {
    const uint32_t n = *n_in;
    uint32_t c_hits = 0, c_paths = 0, c_pmiss = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += stride) {
        const uint32_t qi = base + threadIdx.x;
        bool alive = false;
        uint32_t slot = 0;
        if (qi < n) {
            slot = q_in[qi];
            uint32_t px, py;
            slot_pixel(kp, slot, px, py);
            const float4 o4 = kp.p_o[slot], d4 = kp.p_d[slot], thr4 = kp.p_thr[slot], col4 = kp.p_col[slot];
            uint4 st = kp.p_st[slot], st2 = kp.p_st2[slot];
            const uint2 ms2 = kp.p_ms[slot];
            const float4 tuvo = kp.h_tuvo[slot];
            const uint2 hid = kp.h_id[slot];
            Ray ray{mk(o4.x, o4.y, o4.z), mk(d4.x, d4.y, d4.z)};
            f3 thr = xyz(thr4), col = xyz(col4);
            float acc_rough = o4.w;
            Bounces bounce{st.x, st.y, st.z};
            uint32_t iter = st.w;
            MediumStack ms{uint64_t(ms2.x) | (uint64_t(ms2.y) << 32), int(st2.w)};
            const uint32_t fidx = st2.z;
            Sampler smp{frame_count(kp, fidx), pcg_hash(px + py * kp.Wu), st2.x};
            bool path_alive = false;

            if (tuvo.x < kp.far_) {  // :898
                c_hits++;
                Hit hit;
                hit.t = tuvo.x;
                hit.orient = tuvo.w;
                hit.pos = ray.o + ray.d * hit.t;
                if (hid.x & HG_SPHERE_BIT) {
                    const uint32_t si = hid.x & ~HG_SPHERE_BIT;
                    const float4 cr = kp.spheres[3 * si];
                    hit.n = normalize(hit.pos - xyz(cr)) * hit.orient;
                    hit.mat = __float_as_uint(kp.spheres[3 * si + 1].w);
                } else {
                    const HgDevMesh& md = kp.meshes[hid.y];
                    const float4 n0 = kp.normals[3 * hid.x], d1 = kp.normals[3 * hid.x + 1],
                                 d2 = kp.normals[3 * hid.x + 2];
                    f3 nn = (xyz(n0) + xyz(d1) * tuvo.y) + xyz(d2) * tuvo.z;
                    nn = nn * hit.orient;
                    const float* m = md.w2l;
                    const f3 w = mk(((nn.x * m[0] + nn.y * m[1]) + nn.z * m[2]) + 0.0f * m[3],
                                    ((nn.x * m[4] + nn.y * m[5]) + nn.z * m[6]) + 0.0f * m[7],
                                    ((nn.x * m[8] + nn.y * m[9]) + nn.z * m[10]) + 0.0f * m[11]);
                    hit.n = normalize(w);
                    hit.mat = md.material;
                }
                const Mat mt = load_mat(kp, hit.mat);
                col = col + xyz(mt.emis_rough) * thr;                       // :901-902
                uint32_t bt = 0;
                const f3 att = evaluate_hit(kp, smp, ms, ray, hit, mt, bt);  // :905
                bounce.bump(bt);
                thr = thr * att;                                            // :908
                acc_rough += mt.emis_rough.w * thr.x;                        // :911
                const float rr = smp.get1(ID_RR);                           // :915
                smp.offset += BOUNCE_INC;                                   // :921
                const float contribution = fmaxf(fmaxf(thr.x, thr.y), thr.z);
                if (!(rr > contribution)) {                                 // :930
                    thr = thr * (1.0f / contribution);
                    iter++;
                    // next iteration of :889 only if the loop bound and the bounce limits (:891) allow it
                    path_alive = iter <= kp.max_bounces && !(bounce.diffuse > kp.max_diff ||
                                                            bounce.glossy > kp.max_glossy ||
                                                            bounce.transmission > kp.max_trans);
                }
            } else {
                // the path's camera ray: no bounce accepted yet (iter counts the rays after the first)
                c_pmiss += iter == 0u && bounce.diffuse == 0u && bounce.glossy == 0u && bounce.transmission == 0u;
                col = col + sample_sky(kp, ray.d, sky_level(kp, acc_rough)) * thr;  // :941
            }

            uint32_t sample = st2.y, fi = fidx;
            float4 sum4 = kp.p_sum[slot];
            if (!path_alive) {
                // trace_ray returned: RayColor += result (:1043)
                f3 sum = xyz(sum4) + col;
                sample++;
                bool next = false;
                if (sample < kp.spp) {
                    next = true;  // next sample of the same dispatch: statics persist (:188-189)
                } else {
                    // frame done: Output = RayColor / SPP, then the accumulation blend
                    const float sppf = float(kp.spp);
                    const f3 color = mk(sum.x / sppf, sum.y / sppf, sum.z / sppf);
                    float4 acc = kp.acc[slot];
                    if (kp.accumulate) {
                        const float w = 1.0f / float(smp.frame);
                        const float k = 1.0f - w;
                        acc = make_float4(acc.x * k + color.x * w, acc.y * k + color.y * w, acc.z * k + color.z * w,
                                          acc.w * k + 1.0f * w);
                    } else {
                        acc = make_float4(color.x, color.y, color.z, 1.0f);
                    }
                    kp.acc[slot] = acc;
                    fi++;
                    if (fi < uint32_t(kp.n_frames)) {
                        next = true;  // next frame: a new dispatch, statics reset
                        sample = 0;
                        sum = mk(0, 0, 0);
                        smp.frame = frame_count(kp, fi);
                        smp.offset = 0;
                        ms = MediumStack{0ull, 0};
                    }
                }
                if (next) {
                    ray = camera_ray(kp, smp, (float(px) / kp.W) * 2.0f - 1.0f, (float(py) / kp.H) * 2.0f - 1.0f);
                    thr = mk(1, 1, 1);
                    col = mk(0, 0, 0);
                    acc_rough = 0.0f;
                    bounce = Bounces{0, 0, 0};
                    iter = 0;
                    path_alive = true;
                    c_paths++;
                }
                sum4 = make_float4(sum.x, sum.y, sum.z, 0.0f);
                kp.p_sum[slot] = sum4;
            }
            if (path_alive) {
                kp.p_o[slot] = make_float4(ray.o.x, ray.o.y, ray.o.z, acc_rough);
                kp.p_d[slot] = make_float4(ray.d.x, ray.d.y, ray.d.z, 0.0f);
                kp.p_thr[slot] = make_float4(thr.x, thr.y, thr.z, 0.0f);
                kp.p_col[slot] = make_float4(col.x, col.y, col.z, 0.0f);
                kp.p_st[slot] = make_uint4(bounce.diffuse, bounce.glossy, bounce.transmission, iter);
                kp.p_st2[slot] = make_uint4(smp.offset, sample, fi, uint32_t(ms.sp));
                kp.p_ms[slot] = make_uint2(uint32_t(ms.s), uint32_t(ms.s >> 32));
            }
            alive = path_alive;
        }
        wave_append(alive, slot, q_out, n_out);
    }
    if (kp.counters) {
        const uint32_t v[7] = {c_paths, 0, 0, 0, 0, 0, c_hits};
        wave_add_counters(kp, v);
        const uint32_t pm = wave_sum(c_pmiss);
        if (lane_id() == 0 && pm) atomicAdd(kp.counters + 16, (unsigned long long)pm);
    }
}

// ---------------------------------------------------------------------------------------------------------
// launchers (hg_runtime.hip)
// ---------------------------------------------------------------------------------------------------------
hipError_t hg_wf_launch_gen(const HgKernelParams& kp, uint32_t* q_out, uint32_t* n_out, hipStream_t s) {
    const int grid = int(std::min<uint32_t>((kp.n_slots + 255) / 256, 4096u));
    hipLaunchKernelGGL(hg_wf_gen, dim3(grid), dim3(256), 0, s, kp, q_out, n_out);
    return hipGetLastError();
}

size_t hg_wf_trace_lds_bytes(uint32_t stack_depth, int block) {
    return size_t(std::min<uint32_t>(stack_depth, HG_LDS_STACK)) * size_t(block) * sizeof(uint32_t);
}

hipError_t hg_wf_launch_trace(const HgKernelParams& kp, int grid, int block, bool counters, const uint32_t* q_in,
                              const uint32_t* n_in, uint32_t* head, hipStream_t s) {
    const size_t lds = hg_wf_trace_lds_bytes(kp.stack_depth, block);
    if (counters)
        hipLaunchKernelGGL(hg_wf_trace<true>, dim3(grid), dim3(block), lds, s, kp, q_in, n_in, head);
    else
        hipLaunchKernelGGL(hg_wf_trace<false>, dim3(grid), dim3(block), lds, s, kp, q_in, n_in, head);
    return hipGetLastError();
}

hipError_t hg_wf_launch_shade(const HgKernelParams& kp, int grid, const uint32_t* q_in, const uint32_t* n_in,
                              uint32_t* q_out, uint32_t* n_out, hipStream_t s) {
    hipLaunchKernelGGL(hg_wf_shade, dim3(grid), dim3(256), 0, s, kp, q_in, n_in, q_out, n_out);
    return hipGetLastError();
}

int hg_wf_trace_blocks_per_cu(int block, size_t lds_bytes) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, hg_wf_trace<true>, block, lds_bytes) != hipSuccess) return 1;
    return n > 0 ? n : 1;
}
