// hg_device.h — device-side building blocks of the Halogen hot path shared by the kernels of hg_mega.hip
// (lockstep, regenerating and streaming megakernels, and the render server's persistent form of the streaming one).
//
// Every function restates a piece of the reference (file:line in its comment) in the reference's
// operation order, compiled with -ffp-contract=off and the shared arithmetic spec include/hg_fmath.h, so the
// results are bit-identical to the CPU oracle.
#pragma once
#include <hip/hip_runtime.h>

#include "hg_fmath.h"
#include "hg_layout.h"

#pragma clang fp contract(off)

namespace hgd {

// ---------------------------------------------------------------------------------------------------
// float3 helpers with the reference's evaluation order (no FMA)
// ---------------------------------------------------------------------------------------------------
struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float len(f3 a) { return __builtin_sqrtf(dot(a, a)); }
__device__ __forceinline__ float rcp_exact(float x);
// normalize = v * (1/sqrt(dot(v,v))) (hg_fmath.h hg_rnorm)
__device__ __forceinline__ f3 normalize(f3 a) { return a * hg_rnorm(dot(a, a)); }
__device__ __forceinline__ f3 lerp(f3 a, f3 b, float s) { return a + (b - a) * s; }
__device__ __forceinline__ f3 xyz(float4 v) { return mk(v.x, v.y, v.z); }

// mul(M, float4(v, w)), M given row-major in m[r*4+c] (rows 0..2)
__device__ __forceinline__ f3 xform(const float* m, f3 v, float w) {
    return mk(((m[0] * v.x + m[1] * v.y) + m[2] * v.z) + m[3] * w,
              ((m[4] * v.x + m[5] * v.y) + m[6] * v.z) + m[7] * w,
              ((m[8] * v.x + m[9] * v.y) + m[10] * v.z) + m[11] * w);
}

// ---------------------------------------------------------------------------------------------------
// Sampler (HalogenRandom.hlsl)
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pcg_hash(uint32_t v) {  // u32_hash :110-115
    uint32_t state = v * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
__device__ __forceinline__ uint32_t hash_combine(uint32_t seed, uint32_t v) {  // :131-133
    return seed ^ (v + (seed << 6) + (seed >> 2));
}
// the Laine–Karras-style body of owen_scramble (:154-158), on the already bit-reversed value
__device__ __forceinline__ uint32_t lk_body(uint32_t x, uint32_t seed) {
    x ^= x * 0x3d20adeau;
    x += seed;
    x *= (seed >> 16) | 1u;
    x ^= x * 0x05526c56u;
    x ^= x * 0x53a22864u;
    return x;
}
__device__ __forceinline__ uint32_t brev(uint32_t x) { return __builtin_bitreverse32(x); }
// owen_scramble(v, s) = brev(lk(brev(v), s))
__device__ __forceinline__ uint32_t owen(uint32_t v, uint32_t s) { return brev(lk_body(brev(v), s)); }
// Sobol dimension 1 (Pascal matrix mod 2): bit p (MSB-first) of sobol(i,1) = XOR over set bits k of i
// with k ⊇ p  ->  superset-XOR transform of i, then bit-reversed.
__device__ __forceinline__ uint32_t superset_xor(uint32_t z) {
    z ^= (z >> 1) & 0x55555555u;
    z ^= (z >> 2) & 0x33333333u;
    z ^= (z >> 4) & 0x0F0F0F0Fu;
    z ^= (z >> 8) & 0x00FF00FFu;
    z ^= (z >> 16) & 0x0000FFFFu;
    return z;
}
constexpr float kInv2_32 = 4294967296.0f;

struct Sampler {
    uint32_t frame;   // Sobol index (FrameCount)
    uint32_t pixel;   // pixelID = u32_hash(x + y*W)
    uint32_t offset;  // SobolDimensionOffset
    // float_owen_scrambled_sobol (:252-259): owen(sobol(i,0), pcg(seed)) = brev(lk(i, pcg(seed)))
    __device__ __forceinline__ float get1(uint32_t id) const {
        uint32_t seed = pixel ^ pcg_hash(offset + id);
        return float(brev(lk_body(frame, pcg_hash(seed)))) / kInv2_32;
    }
    // float2_owen_scrambled_sobol (:261-268, :215-228)
    __device__ __forceinline__ void get2(uint32_t id, float& a, float& b) const {
        uint32_t seed = pixel ^ pcg_hash(offset + id);
        uint32_t sh = owen(frame, seed);  // shuffled index
        a = float(brev(lk_body(sh, hash_combine(seed, 0u)))) / kInv2_32;
        b = float(brev(lk_body(superset_xor(sh), hash_combine(seed, 1u)))) / kInv2_32;
    }
};

constexpr uint32_t ID_FOCAL = 0, ID_JITTER = 1, ID_ROUGH = 2, ID_PROPERTY = 3, ID_RR = 4, BOUNCE_INC = 5;
#define HLSL_PI (180.0f * HG_DEG2RAD)

// ---------------------------------------------------------------------------------------------------
// Per-lane path state
// ---------------------------------------------------------------------------------------------------
struct Counters {
    uint32_t rays, tri, aabb, node_rounds, tri_rounds, hits;  // *_rounds: wave-level loop iterations (one lane counts)
    uint32_t shade_rounds;
    uint32_t primary_miss;  // camera rays that hit nothing
};
// 1 in exactly one active lane (the lowest): summed over lanes, counts the wave-level executions of a code point
// Wave clock (s_memtime) for the counting instantiations' phase split; volatile + memory clobber keep the
// compiler from moving it across the code it brackets.
__device__ __forceinline__ uint64_t wave_clock() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
    return t;
}
// 64-lane ballot of a bool straight from the compare mask (the HIP __ballot(int) materialises the predicate in a
// VGPR and compares it again)
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t wave_count(bool p) { return uint32_t(__builtin_popcountll(wave_ballot(p))); }
__device__ __forceinline__ uint32_t wave_once() {
    return __lane_id() == uint32_t(__builtin_ctzll(__ballot(1))) ? 1u : 0u;
}

// bounceTypes[3] of trace_ray (:887) kept as three named registers (a runtime-indexed array would go to
// scratch memory on gfx950)
struct Bounces {
    uint32_t diffuse, glossy, transmission;
    __device__ __forceinline__ void bump(uint32_t t) {
        diffuse += t == 0u;
        glossy += t == 1u;
        transmission += t == 2u;
    }
};

struct Ray {
    f3 o, d;
};

struct Hit {
    float t;
    float orient;
    f3 pos, n;
    uint32_t mat;
};

// nested-dielectric stack (:188-189): 8 material indices packed one byte each in a u64 (the medium of a
// stack entry is always the internal medium of a material, so its index identifies it completely)
struct MediumStack {
    uint64_t s;
    int sp;
    __device__ __forceinline__ uint32_t get(int i) const { return uint32_t(s >> (8 * i)) & 0xFFu; }
};

// material record accessors
struct Mat {
    float4 albedo, spec_metal, emis_rough, absorb_ior, prio_id_r2;
};
__device__ __forceinline__ Mat load_mat(const HgKernelParams& kp, uint32_t m) {
    const float4* p = kp.materials + 5 * m;
    return Mat{p[0], p[1], p[2], p[3], p[4]};
}
__device__ __forceinline__ int32_t mat_priority(const HgKernelParams& kp, uint32_t m) {
    return __float_as_int(kp.materials[5 * m + 4].x);
}

// ---------------------------------------------------------------------------------------------------
// Intersection (:244-485)
// ---------------------------------------------------------------------------------------------------
// 1/x, correctly rounded (the reference's `1 / det`, `1 / dir` in IEEE fp32).  With HG_FAST_RCP the hardware
// reciprocal (<= 1 ulp) is refined by one FMA Newton step, correctly rounded for every x whose exponent keeps x
// and 1/x normal (checked for all 2^32 inputs by hg_selftest, tests/test_gpu_selftest.py); zeros, denormals,
// huge values, infinities and NaNs take the IEEE division.
__device__ __forceinline__ float rcp_exact(float x) {
#if HG_FAST_RCP
    const uint32_t ex = (__float_as_uint(x) >> 23) & 0xFFu;
    if (__builtin_expect(ex - 2u <= 250u, 1)) {
        const float r = __builtin_amdgcn_rcpf(x);
        const float e = __builtin_fmaf(-x, r, 1.0f);
        return __builtin_fmaf(e, r, r);
    }
#endif
    return 1.0f / x;
}

// (first triangle, count) of a leaf ref (hg_layout.h): inline for small leaves, else from the leaf table
__device__ __forceinline__ uint2 leaf_range(const HgKernelParams& kp, uint32_t ref);

// base + 32-bit byte offset: lets the compiler use the scalar-base + VGPR-offset load form (upload keeps every
// scene array below 4 GiB, hg_runtime.hip)
template <class T>
__device__ __forceinline__ T ld_off(const T* base, uint32_t byte_off) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}

// Frame colour of launch frame f (0 .. n_frames-1) for accumulator slot `slot`: [slot][frame], one pixel's frames
// contiguous (hg_blend_frames* read the same layout)
__device__ __forceinline__ size_t fc_slot_frame(size_t slot, uint32_t f, uint32_t n_frames) {
    return slot * size_t(n_frames) + f;
}
// Frame colours are written once by the trace and read once by the blend: both go through the non-temporal hint, so
// the 2.1 GB a 64-frame C3 launch writes is not kept in L2 ahead of the BVH lines (+0.2..0.6 %, sweep_r03_n)
__device__ __forceinline__ void fc_store(float4* p, float4 v) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z);
    __builtin_nontemporal_store(v.w, &p->w);
}
__device__ __forceinline__ float4 fc_load(const float4* p) {
    return make_float4(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y),
                       __builtin_nontemporal_load(&p->z), __builtin_nontemporal_load(&p->w));
}
__device__ __forceinline__ size_t fc_index(const HgKernelParams& kp, uint32_t f, size_t slot) {
    return fc_slot_frame(slot, f, uint32_t(kp.n_frames));
}

// Triangle ti's Moller-Trumbore operands from its packed 36-B record (v0, e1, e2): a = (v0, e1.x), b = (e1.yz, e2.xy),
// cz = e2.z, as two 4-B-aligned 16-B loads and one 4-B load.  (The three SoA streams of rounds 1-2 put a leaf's
// triangles on 3-5 lines instead of 2-3: L1 misses -20 % with this record; 48-B padded records lost 0.3-5.7 %; the
// non-temporal hint on these loads lost 10 %, a leaf's triangles are re-read by the next rounds and waves.)
__device__ __forceinline__ void tri_load(const HgKernelParams& kp, uint32_t ti, float4& a, float4& b, float& cz) {
    typedef float hg_v4u __attribute__((ext_vector_type(4), aligned(4)));  // 4-B aligned 16-B loads
    const char* p = reinterpret_cast<const char*>(kp.tris) + ti * 36u;
    const hg_v4u va = *reinterpret_cast<const hg_v4u*>(p), vb = *reinterpret_cast<const hg_v4u*>(p + 16);
    a = make_float4(va.x, va.y, va.z, va.w);
    b = make_float4(vb.x, vb.y, vb.z, vb.w);
    cz = *reinterpret_cast<const float*>(p + 32);
}

// Load of scene data the kernel never writes (mesh records, spheres) through the constant address space: a
// wave-uniform address then compiles to a scalar load (s_load_dwordx4, scalar cache) even after the kernel's own
// global stores, where a generic load must stay a vector load (one full memory latency per mesh / sphere).
typedef float hg_v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldc(const float4* base, uint32_t i) {
    typedef const __attribute__((address_space(4))) hg_v4f* cptr;
    const hg_v4f v = ((cptr)(uintptr_t)base)[i];
    return make_float4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint2 leaf_range(const HgKernelParams& kp, uint32_t ref) {
    const uint32_t cnt = (ref >> HG_LEAF_CNT_SHIFT) & HG_LEAF_INLINE_MAX;
    if (__builtin_expect(cnt != 0u, 1)) return make_uint2(ref & HG_LEAF_PAYLOAD, cnt);
    return ld_off(kp.leaves, (ref & HG_LEAF_PAYLOAD) << 3);
}

__device__ __forceinline__ float ray_aabb(f3 A, f3 B, f3 o, f3 inv) {  // :244-259
    f3 t1 = (A - o) * inv;
    f3 t2 = (B - o) * inv;
    float tMin = fminf(t1.x, t2.x);
    float tMax = fmaxf(t1.x, t2.x);
    tMin = fmaxf(tMin, fminf(t1.y, t2.y));
    tMax = fminf(tMax, fmaxf(t1.y, t2.y));
    tMin = fmaxf(tMin, fminf(t1.z, t2.z));
    tMax = fminf(tMax, fmaxf(t1.z, t2.z));
    return tMax > fmaxf(0.0f, tMin) ? tMin : HG_INF;
}

// A child-pair record (hg_runtime.hip, BLAS pass 2): both children's boxes and refs in 64 B, 56 of them used:
// q0 = (A.lo, refA), q1 = (A.hi, refB), q2 = (B.lo, -), q3 = (B.hi, -).  (The coordinate-by-coordinate form for packed
// FP32 box tests cost 8-16 B of scratch and lost 1-2.4 %)
struct NodePair {
    float4 q0, q1, q2, q3;
};
__device__ __forceinline__ NodePair node_pair(const HgKernelParams& kp, uint32_t node) {
    const uint32_t ro = node << 6;
    return NodePair{ld_off(kp.nodes, ro), ld_off(kp.nodes, ro + 16), ld_off(kp.nodes, ro + 32), ld_off(kp.nodes, ro + 48)};
}
__device__ __forceinline__ uint32_t pair_ref_a(const NodePair& r) { return __float_as_uint(r.q0.w); }
__device__ __forceinline__ uint32_t pair_ref_b(const NodePair& r) { return __float_as_uint(r.q1.w); }
// ray_aabb (:244-259) of both children: dA, dB
__device__ __forceinline__ void pair_dist(const NodePair& r, f3 o, f3 inv, float& dA, float& dB) {
    dA = ray_aabb(xyz(r.q0), xyz(r.q1), o, inv);
    dB = ray_aabb(xyz(r.q2), xyz(r.q3), o, inv);
}

// Returns the closest accepted sphere as index | (orientation < 0) << 31 (HG_NONE if none), its distance in t;
// position/normal/material are resolved after the mesh pass (resolve_sphere), with the same arithmetic.
__device__ uint32_t isect_spheres(const HgKernelParams& kp, const Ray& ray, float& t) {  // :357-376
    float closest = t;
    uint32_t best = HG_NONE;
    f3 inv = mk(rcp_exact(ray.d.x), rcp_exact(ray.d.y), rcp_exact(ray.d.z));
    for (int i = 0; i < kp.n_spheres; ++i) {
        const float4 cr = ldc(kp.spheres, 3 * i);
        const float4 am = ldc(kp.spheres, 3 * i + 1);
        const float4 b = ldc(kp.spheres, 3 * i + 2);
        if (!(ray_aabb(xyz(am), xyz(b), ray.o, inv) < kp.far_)) continue;
        // sphere_intersection :266-303
        f3 center = xyz(cr);
        f3 sh = ray.o - center;
        float bq = 2.0f * dot(sh, ray.d);
        float cq = dot(sh, sh) - cr.w * cr.w;
        float disc = bq * bq - 4.0f * cq;
        if (!(disc >= 0.0f)) continue;  // rayT = INF: never accepted
        float hd = (-bq - __builtin_sqrtf(disc)) / 2.0f;
        uint32_t back = 0;
        if (hd < 0.0f) {
            hd = (-bq + __builtin_sqrtf(disc)) / 2.0f;
            back = 0x80000000u;
        }
        if (hd < closest && hd > 0.0001f) {
            closest = hd;
            best = uint32_t(i) | back;
        }
    }
    t = closest;
    return best;
}
__device__ __forceinline__ void resolve_sphere(const HgKernelParams& kp, const Ray& ray, uint32_t ref, Hit& h) {
    const uint32_t i = ref & 0x7FFFFFFFu;
    const float orient = (ref & 0x80000000u) ? -1.0f : 1.0f;
    const float4 cr = kp.spheres[3 * i];
    h.orient = orient;
    h.pos = ray.o + ray.d * h.t;
    h.n = normalize(h.pos - xyz(cr)) * orient;
    h.mat = __float_as_uint(kp.spheres[3 * i + 1].w);
}

// Exact mesh skip (HgDevMesh::cull_*): bit m of the result is clear when the ray certainly misses both children of
// mesh m's root in the reference's local-space test, or meets them only beyond `best_t` — the reference would test
// those two boxes, push nothing and find nothing there.  Meshes >= 64 are never culled.
__device__ __forceinline__ uint64_t mesh_live_mask(const HgKernelParams& kp, f3 wo, f3 winv, float best_t,
                                                   uint32_t& culled) {
    uint64_t live = ~0ull;
    const float lim = best_t * 1.0001f + 1e-4f;
    const int ncull = kp.n_meshes < 64 ? kp.n_meshes : 64;
    static_assert(sizeof(HgDevMesh) % 16 == 0 && offsetof(HgDevMesh, cull_a_lo) % 16 == 0, "float4 records");
    const float4* mrec = reinterpret_cast<const float4*>(kp.meshes);
    constexpr uint32_t kRec = sizeof(HgDevMesh) / 16, kCull = offsetof(HgDevMesh, cull_a_lo) / 16;
    for (int m = 0; m < ncull; ++m) {
        const float4 hdr = ldc(mrec, m * kRec + kCull - 1);  // root_ref, tri_offset, material, cullable
        if (!__float_as_uint(hdr.w)) continue;
        const float4 alo = ldc(mrec, m * kRec + kCull), ahi = ldc(mrec, m * kRec + kCull + 1),
                     blo = ldc(mrec, m * kRec + kCull + 2), bhi = ldc(mrec, m * kRec + kCull + 3);
        const float dA = ray_aabb(xyz(alo), xyz(ahi), wo, winv);
        const float dB = ray_aabb(xyz(blo), xyz(bhi), wo, winv);
        const bool farA = dA == HG_INF || dA > lim, farB = dB == HG_INF || dB > lim;  // NaN never skips
        if (farA && farB) {
            live &= ~(1ull << m);
            culled++;
        }
    }
    return live;
}

// Triangle test of triangle_intersection_doublesided (:307-355) with every term computed and one combined accept
// (same values as the early-out form).  Returns true when the hit is accepted as the new closest (:416).
// kFlat (the distributed leaf test, measured: stream C3 +0.7 %; the regenerating kernel's sequential loop loses
// 1.5-3 % with it, tools/sweeps/NOTES_r02.md) evaluates the accept without short-circuit branches.
template <bool kFlat = false>
__device__ __forceinline__ bool tri_accept(f3 lo, f3 ld, float4 a, float4 b, float cz, float best_t, float& t,
                                           float& U, float& V, bool& front) {
    const f3 e1 = mk(a.w, b.x, b.y);
    const f3 e2 = mk(b.z, b.w, cz);
    const f3 pvec = cross(ld, e2);
    const float det = dot(pvec, e1);
    const float inv_det = rcp_exact(det);
    const f3 tvec = lo - xyz(a);
    U = dot(tvec, pvec) * inv_det;
    const f3 qvec = cross(tvec, e1);
    V = dot(ld, qvec) * inv_det;
    t = dot(e2, qvec) * inv_det;
    front = det > 0.0f;
    if (kFlat)  // bitwise & of the conditions: one straight compare chain instead of a branch per short-circuit step
        return bool(int(!(fabsf(det) < 0.00000001f)) & int(!(U < 0.0f || U > 1.0f)) & int(!(V < 0.0f || U + V > 1.0f)) &
                    int(t > 0.0f) & int(t > 0.0001f) & int(t < best_t));
    return !(fabsf(det) < 0.00000001f) && !(U < 0.0f || U > 1.0f) && !(V < 0.0f || U + V > 1.0f) && t > 0.0f &&
           t > 0.0001f && t < best_t;
}

// Traversal stack: the first kLds entries of each lane live in LDS ([depth][lane], conflict-free), deeper entries
// (rare: the BLAS depth cap is 32) spill to a per-lane global column, so the LDS footprint does not cap occupancy.
// The LDS part is addressed through the address-space-3 array itself (a generic pointer here would turn every
// access into a flat instruction).
extern __shared__ __attribute__((aligned(16))) uint32_t hg_lds_stack[];
template <uint32_t kLds>
struct Stack {
    uint32_t lane;    // this lane's LDS column
    uint32_t lds_stride;
    uint32_t* spill;  // this lane's spill column
    uint32_t spill_stride;
    __device__ __forceinline__ void store(uint32_t slot, uint32_t v) const {
        if (__builtin_expect(slot < kLds, 1)) hg_lds_stack[__umul24(slot, lds_stride) + lane] = v;  // full-rate mad24
        else spill[(slot - kLds) * spill_stride] = v;
    }
    __device__ __forceinline__ uint32_t load(uint32_t slot) const {
        if (__builtin_expect(slot < kLds, 1)) return hg_lds_stack[__umul24(slot, lds_stride) + lane];
        uint32_t v = spill[(slot - kLds) * spill_stride];
        asm volatile("" : "+v"(v));  // keeps the two loads apart (merged, they become one flat load)
        return v;
    }
    __device__ __forceinline__ void push(uint32_t& sp, uint32_t v) const { store(sp++, v); }
    __device__ __forceinline__ uint32_t pop(uint32_t& sp) const { return load(--sp); }
};
using MegaStack = Stack<HG_MEGA_LDS_STACK>;

// Row-major per-lane LDS layout of a one-wave workgroup (the streaming kernel): word (row, lane) = row * 64 + lane.
// Every access is the lane's one base address plus a compile-time row offset (a ds_read / ds_write immediate), so no
// per-variable LDS addresses occupy registers.
template <uint32_t kRow>
struct RowVec3 {  // a float3 in rows kRow .. kRow+2
    uint32_t lane;
    __device__ __forceinline__ f3 get() const {
        return mk(__uint_as_float(hg_lds_stack[kRow * 64u + lane]), __uint_as_float(hg_lds_stack[(kRow + 1) * 64u + lane]),
                  __uint_as_float(hg_lds_stack[(kRow + 2) * 64u + lane]));
    }
    __device__ __forceinline__ void set(f3 v) const {
        hg_lds_stack[kRow * 64u + lane] = __float_as_uint(v.x);
        hg_lds_stack[(kRow + 1) * 64u + lane] = __float_as_uint(v.y);
        hg_lds_stack[(kRow + 2) * 64u + lane] = __float_as_uint(v.z);
    }
};
template <uint32_t kRow>
struct RowVec4 {  // a float4 in rows kRow .. kRow+3
    uint32_t lane;
    __device__ __forceinline__ float4 get() const {
        return make_float4(__uint_as_float(hg_lds_stack[kRow * 64u + lane]),
                           __uint_as_float(hg_lds_stack[(kRow + 1) * 64u + lane]),
                           __uint_as_float(hg_lds_stack[(kRow + 2) * 64u + lane]),
                           __uint_as_float(hg_lds_stack[(kRow + 3) * 64u + lane]));
    }
    __device__ __forceinline__ void set(float4 v) const {
        hg_lds_stack[kRow * 64u + lane] = __float_as_uint(v.x);
        hg_lds_stack[(kRow + 1) * 64u + lane] = __float_as_uint(v.y);
        hg_lds_stack[(kRow + 2) * 64u + lane] = __float_as_uint(v.z);
        hg_lds_stack[(kRow + 3) * 64u + lane] = __float_as_uint(v.w);
    }
};
// The traversal stack in rows kRow .. kRow+kLds-1 (entry k of the lane at row kRow + k), deeper entries in the lane's
// global spill column, as Stack.
template <uint32_t kLds, uint32_t kRow>
struct RowStack {
    uint32_t lane;
    uint32_t* spill;
    uint32_t spill_stride;
    __device__ __forceinline__ void store(uint32_t slot, uint32_t v) const {
        if (__builtin_expect(slot < kLds, 1)) hg_lds_stack[(kRow + slot) * 64u + lane] = v;
        else spill[(slot - kLds) * spill_stride] = v;
    }
    __device__ __forceinline__ uint32_t load(uint32_t slot) const {
        if (__builtin_expect(slot < kLds, 1)) return hg_lds_stack[(kRow + slot) * 64u + lane];
        uint32_t v = spill[(slot - kLds) * spill_stride];
        asm volatile("" : "+v"(v));
        return v;
    }
    __device__ __forceinline__ void push(uint32_t& sp, uint32_t v) const { store(sp++, v); }
    __device__ __forceinline__ uint32_t pop(uint32_t& sp) const { return load(--sp); }
};

// first mesh index >= m whose cull bit is set (meshes >= 64 carry no bit and are always live); n if none
__device__ __forceinline__ uint32_t next_live_mesh(uint64_t live, uint32_t m, uint32_t n) {
    uint32_t r = 64u;
    if (m < 64u) {
        const uint64_t b = live & (~0ull << m);
        if (b) r = uint32_t(__builtin_ctzll(b));
    } else {
        r = m;
    }
    return r < n ? r : n;
}

// The wave's LDS copy of the mesh records (HG_MESH_LDS): mesh m's first HG_MESH_LDS_F4 float4 (w2l columns, header)
// at float4 index m * HG_MESH_LDS_F4 from word kp.mesh_lds_word (after the kernel's stack rows, hg_mega.hip).
template <bool kLds>
__device__ __forceinline__ float4 mesh_f4(const HgKernelParams& kp, uint32_t m, uint32_t k) {
    if constexpr (kLds) return reinterpret_cast<const float4*>(hg_lds_stack + kp.mesh_lds_word)[m * HG_MESH_LDS_F4 + k];
    else return reinterpret_cast<const float4*>(kp.meshes + m)[k];
}
// copy every mesh record's first HG_MESH_LDS_F4 float4 into the wave's LDS (one wave per workgroup)
__device__ __forceinline__ void mesh_lds_fill(const HgKernelParams& kp, uint32_t lane) {
    float4* mt = reinterpret_cast<float4*>(hg_lds_stack + kp.mesh_lds_word);
    const uint32_t nf4 = uint32_t(kp.n_meshes) * HG_MESH_LDS_F4;
    for (uint32_t i = lane; i < nf4; i += 64u) {
        const uint32_t m = i / HG_MESH_LDS_F4;
        mt[i] = reinterpret_cast<const float4*>(kp.meshes + m)[i - m * HG_MESH_LDS_F4];
    }
}

// world -> local ray of mesh m, direction NOT normalized (:390-392), its reciprocal and the root ref
template <bool kLds = false>
__device__ __forceinline__ void mesh_local_ray(const HgKernelParams& kp, const Ray& ray, uint32_t m, f3& lo, f3& ld,
                                               f3& inv, uint32_t& root) {
    const float4 c0 = mesh_f4<kLds>(kp, m, 0), c1 = mesh_f4<kLds>(kp, m, 1), c2 = mesh_f4<kLds>(kp, m, 2),
                 c3 = mesh_f4<kLds>(kp, m, 3);  // worldToLocal columns
    root = __float_as_uint(mesh_f4<kLds>(kp, m, 4).x);
    lo = mk(((c0.x * ray.o.x + c1.x * ray.o.y) + c2.x * ray.o.z) + c3.x * 1.0f,
            ((c0.y * ray.o.x + c1.y * ray.o.y) + c2.y * ray.o.z) + c3.y * 1.0f,
            ((c0.z * ray.o.x + c1.z * ray.o.y) + c2.z * ray.o.z) + c3.z * 1.0f);
    ld = mk(((c0.x * ray.d.x + c1.x * ray.d.y) + c2.x * ray.d.z) + c3.x * 0.0f,
            ((c0.y * ray.d.x + c1.y * ray.d.y) + c2.y * ray.d.z) + c3.y * 0.0f,
            ((c0.z * ray.d.x + c1.z * ray.d.y) + c2.z * ray.d.z) + c3.z * 0.0f);
    inv = mk(rcp_exact(ld.x), rcp_exact(ld.y), rcp_exact(ld.z));
}

// Accepted mesh hit (:452-471): interpolated normal x orientation through the inverse-transpose, hit position.
template <bool kLds = false>
__device__ __forceinline__ void resolve_mesh(const HgKernelParams& kp, const Ray& ray, float best_t, float best_u,
                                             float best_v, uint32_t best_tri, uint32_t best_mesh, Hit& h) {
    const uint32_t tri = best_tri & 0x7FFFFFFFu;
    const float orient = (best_tri & 0x80000000u) ? -1.0f : 1.0f;
    h.t = best_t;
    h.mat = __float_as_uint(mesh_f4<kLds>(kp, best_mesh, 4).z);  // HgDevMesh::material
    h.orient = orient;
    const float4 n0 = kp.normals[3 * tri], d1 = kp.normals[3 * tri + 1], d2 = kp.normals[3 * tri + 2];
    f3 n = (xyz(n0) + xyz(d1) * best_u) + xyz(d2) * best_v;
    n = n * orient;
    // mul(float4(n,0), worldToLocal): row vector times matrix (inverse-transpose normal transform); w2l is column-major,
    // so m[4c + r] = column c, row r and the dot products run down the columns
    const float4 m0 = mesh_f4<kLds>(kp, best_mesh, 0), m1 = mesh_f4<kLds>(kp, best_mesh, 1),
                 m2 = mesh_f4<kLds>(kp, best_mesh, 2);
    f3 w = mk(((n.x * m0.x + n.y * m0.y) + n.z * m0.z) + 0.0f * m0.w,
              ((n.x * m1.x + n.y * m1.y) + n.z * m1.z) + 0.0f * m1.w,
              ((n.x * m2.x + n.y * m2.y) + n.z * m2.z) + 0.0f * m2.w);
    h.n = normalize(w);
    h.pos = ray.o + ray.d * best_t;
}

// ---- wave-wide inclusive scans over 64 lanes (DPP row shifts + row broadcasts, the GFX9 form); every lane of the
// wave must be active
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_(uint32_t x) {
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), kCtrl, kRowMask, 0xF, false));  // invalid source: 0
}
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
    x += dpp_<0x111, 0xF>(x);  // row_shr:1
    x += dpp_<0x112, 0xF>(x);  // row_shr:2
    x += dpp_<0x114, 0xF>(x);  // row_shr:4
    x += dpp_<0x118, 0xF>(x);  // row_shr:8
    x += dpp_<0x142, 0xA>(x);  // row_bcast:15 into rows 1 and 3
    x += dpp_<0x143, 0xC>(x);  // row_bcast:31 into rows 2 and 3
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    x = max(x, dpp_<0x111, 0xF>(x));
    x = max(x, dpp_<0x112, 0xF>(x));
    x = max(x, dpp_<0x114, 0xF>(x));
    x = max(x, dpp_<0x118, 0xF>(x));
    x = max(x, dpp_<0x142, 0xA>(x));
    x = max(x, dpp_<0x143, 0xC>(x));
    return x;
}
// Lanes of one wave exchanging data through LDS: the fences make the other lanes' LDS writes visible to this lane's
// later reads (and keep the compiler from forwarding its own stores across them).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-wave LDS scratch of the distributed leaf test (HG_LEAF_DIST): per lane, the best (t bits << 32 | triangle)
// key found for its ray, and one word of the owner table.  3 words per lane.
constexpr uint32_t kLeafShareWords = 3;
struct LeafShare {
    uint32_t w;  // word offset of this wave's 192-word region (even: the keys are u64)
    __device__ __forceinline__ unsigned long long* key(uint32_t i) const {
        return reinterpret_cast<unsigned long long*>(hg_lds_stack + w) + i;
    }
    __device__ __forceinline__ uint32_t& tab(uint32_t i) const { return hg_lds_stack[w + 128u + i]; }
};

__device__ __forceinline__ float bperm_f(int addr, float x) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(x)));
}

// Distributed leaf test (HG_LEAF_DIST; HC:404-420): the triangles of every lane's current leaf form (ray, triangle)
// pairs numbered lane by lane (a wave prefix sum of the leaf sizes), and each round all 64 lanes test 64 of them.
// A pair's lane finds its owner through a per-wave table (the owner's lane id stored at the pair index where its
// run starts, then a running max over the lanes), fetches the owner's local ray and best_t by ds_bpermute, and
// folds an accepted hit into the owner's key (t bits << 32 | triangle) with an LDS 64-bit atomic min.  After each
// round an owner whose key came from that round pulls u, v and the facing from the winning pair's lane.
// Exact: in the reference's sequential loop every acceptance condition but `t < closest` is independent of the
// other triangles, and `closest` only falls, so the loop ends on the first triangle (in leaf order) of minimal t
// among those with t < best_t at the leaf's start.  t > 1e-4 is positive, so its bit pattern orders like its
// value, and the lower triangle index wins a tie: the key minimum is that triangle.  Counters are the same
// (one triangle test per pair).
// Precondition: every lane of the wave is active (the DPP scans and ds_bpermute read other lanes' registers; under a
// partial EXEC a disabled lane's register is stale and the prefix sums skip it).  The streaming kernel meets it by
// construction: trav_step runs at the top level of loops whose exits are wave-uniform (ballot counts).  Debug builds
// (HG_CHECK_EXEC=1) check it and take the sequential leaf loop when a lane is off (returns false); the check is
// compiled out of the product build because keeping the fallback loop live costs the kernel 16 B/lane of scratch.
struct LeafRay {  // the lane's side of a leaf test: its mesh-local ray and running best hit
    const f3& lo;
    const f3& ld;
    float& best_t;
    float& best_u;
    float& best_v;
    uint32_t& best_tri;
    uint32_t& best_mesh;
    uint32_t mi;
};
__device__ __forceinline__ bool leaf_dist(const HgKernelParams& kp, const LeafRay& t, Counters& c, const LeafShare& ls,
                                          uint32_t first, uint32_t n) {
#if HG_CHECK_EXEC
    if (__ballot(1) != ~0ull) {  // partial EXEC: the sequential loop instead (see above), counted in counter slot 17
        if (kp.counters) atomicAdd(kp.counters + 17, 1ull);
        return false;
    }
#endif
    const uint32_t lane = __lane_id();
    const uint32_t incl = wave_incl_add(n);
    const uint32_t total = uint32_t(__builtin_amdgcn_readlane(int(incl), 63));
    if (total == 0u) return true;
    const uint32_t start = incl - n;
    const uint32_t fo = first - start;  // owner's triangle index = fo + pair index (mod 2^32)
    if (n) *ls.key(lane) = ~0ull;
    for (uint32_t base = 0; base < total; base += 64u) {
        c.tri_rounds += wave_once();
        ls.tab(lane) = 0u;
        wave_lds_sync();
        if (n && start < base + 64u && incl > base) ls.tab(start > base ? start - base : 0u) = lane + 1u;
        wave_lds_sync();
        const uint32_t o = wave_incl_max(ls.tab(lane)) - 1u;  // owner lane of pair base + lane
        const int addr = int(o << 2);
        const f3 olo = mk(bperm_f(addr, t.lo.x), bperm_f(addr, t.lo.y), bperm_f(addr, t.lo.z));
        const f3 old = mk(bperm_f(addr, t.ld.x), bperm_f(addr, t.ld.y), bperm_f(addr, t.ld.z));
        const float obt = bperm_f(addr, t.best_t);
        const uint32_t ti = uint32_t(__builtin_amdgcn_ds_bpermute(addr, int(fo))) + base + lane;
        bool acc = false;
        float tt = 0.0f, U = 0.0f, V = 0.0f;
        bool front = false;
        if (base + lane < total) {
            float4 a, b;
            float cz;
            tri_load(kp, ti, a, b, cz);
            c.tri++;
            acc = tri_accept<true>(olo, old, a, b, cz, obt, tt, U, V, front);
        }
        wave_lds_sync();
        if (acc) atomicMin(ls.key(o), (static_cast<unsigned long long>(__float_as_uint(tt)) << 32) | ti);
        wave_lds_sync();
        // owners: did this round's pairs improve the key?  Then pull u, v, facing from the winning pair's lane.
        unsigned long long k = ~0ull;
        if (n) k = *ls.key(lane);
        const uint32_t wp = uint32_t(k) - fo - base;  // winning pair's lane, when it is in this round
        const bool mine = n && k != ~0ull && wp < 64u && uint32_t(k) - fo < total;
        const int src = int((wp & 63u) << 2);
        const float wu = bperm_f(src, U), wv = bperm_f(src, V);
        const uint32_t wf = uint32_t(__builtin_amdgcn_ds_bpermute(src, front ? 1 : 0));
        if (mine) {
            t.best_t = __uint_as_float(uint32_t(k >> 32));
            t.best_u = wu;
            t.best_v = wv;
            t.best_tri = uint32_t(k) | (wf ? 0u : 0x80000000u);
            t.best_mesh = t.mi;
        }
    }
    return true;
}

// get_ray_scene_intersection_mesh, :378-472.
// Per-lane mesh cursor: each lane walks its own live meshes in buffer order (the reference's order, so ties resolve
// identically) and moves to its next mesh as soon as it finishes one, so a wave waits for the lane with the most total
// work instead of the slowest lane of every mesh in turn.  Inside a mesh the traversal keeps the current node in a
// register (the reference's push-near-then-pop-near is a no-op on order) and runs a relaxed while-while: the lanes
// descend inner nodes together while more than kp.descent_t of them are still descending (0: until every lane is at a
// leaf), and in any case until at least one lane can make other progress; then each tests its leaf.  Each lane's own
// sequence of node / leaf steps is the reference's.
template <bool kMeshLds = false, class Stk>
__device__ bool isect_meshes(const HgKernelParams& kp, const Ray& ray, Hit& h, Counters& c, const Stk& stk) {
    const float eps = 0.0001f;
    float best_t = h.t;  // closestIntersection.rayT starts at the sphere hit (:381)
    float best_u = 0.0f, best_v = 0.0f;
    uint32_t best_tri = HG_NONE;  // global triangle index | (orientation < 0) << 31
    uint32_t best_mesh = 0;
    uint32_t culled = 0;
    const f3 winv = mk(rcp_exact(ray.d.x), rcp_exact(ray.d.y), rcp_exact(ray.d.z));
    const uint64_t live = mesh_live_mask(kp, ray.o, winv, best_t, culled);
    c.aabb += 2 * culled;
    const uint32_t nm = uint32_t(kp.n_meshes);
    uint32_t mi = next_live_mesh(live, 0u, nm);
    bool active = mi < nm;
    f3 lo = mk(0, 0, 0), ld = mk(0, 0, 0), inv = mk(0, 0, 0);
    uint32_t node = HG_NONE, sp = 0;
    if (active) mesh_local_ray<kMeshLds>(kp, ray, mi, lo, ld, inv, node);
    while (__any(active)) {
        const uint64_t act_mask = wave_ballot(active);
        const uint32_t dt = kp.descent_t;
        for (uint64_t dm = act_mask & wave_ballot(int32_t(node) >= 0);
             dm != 0ull && (uint32_t(__builtin_popcountll(dm)) > dt || dm == act_mask);
             dm = act_mask & wave_ballot(int32_t(node) >= 0)) {
            c.node_rounds += wave_once();
            if (active && int32_t(node) >= 0) {
                const NodePair np = node_pair(kp, node);
                float dA, dB;
                pair_dist(np, lo, inv, dA, dB);
                c.aabb += 2;
                const uint32_t refA = pair_ref_a(np), refB = pair_ref_b(np);
                // reference (:430-444): push far, push near (each only if tEntry < closest), pop near
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
        if (active && node != HG_NONE && (node & HG_LEAF_BIT)) {  // a leaf: its triangles in order (:404-420)
            const uint2 leaf = leaf_range(kp, node);
            const uint32_t end = leaf.x + leaf.y;
            for (uint32_t ti = leaf.x; ti < end; ++ti) {
                c.tri_rounds += wave_once();
                float4 a, b;
                float cz;
                tri_load(kp, ti, a, b, cz);
                c.tri++;
                float t, U, V;
                bool front;
                if (tri_accept(lo, ld, a, b, cz, best_t, t, U, V, front)) {
                    best_t = t;
                    best_u = U;
                    best_v = V;
                    best_tri = ti | (front ? 0u : 0x80000000u);
                    best_mesh = mi;
                }
            }
            node = sp > 0 ? stk.pop(sp) : HG_NONE;
        }
        if (active && node == HG_NONE) {  // this mesh is done: the lane's next live mesh
            mi = next_live_mesh(live, mi + 1u, nm);
            if (mi < nm) mesh_local_ray<kMeshLds>(kp, ray, mi, lo, ld, inv, node);
            else active = false;
        }
    }
    // :452-471
    if (best_t < (h.t - eps) && best_t < kp.far_) {
        resolve_mesh<kMeshLds>(kp, ray, best_t, best_u, best_v, best_tri, best_mesh, h);
        return true;
    }
    return false;
}

template <bool kMeshLds = false, class Stk>
__device__ __forceinline__ Hit intersect(const HgKernelParams& kp, const Ray& ray, Counters& c, const Stk& stk) {  // get_ray_intersection :474-485
    Hit h;
    h.t = HG_INF;
    h.orient = 0.0f;
    h.pos = mk(0, 0, 0);
    h.n = mk(0, 0, 0);
    h.mat = 0;
    c.rays++;
    const uint32_t sph = isect_spheres(kp, ray, h.t);
    if (!isect_meshes<kMeshLds>(kp, ray, h, c, stk) && sph != HG_NONE) resolve_sphere(kp, ray, sph, h);
    return h;
}

// ---------------------------------------------------------------------------------------------------
// Resumable get_ray_intersection (:474-485) for the streaming kernel: the same spheres / exact mesh cull /
// per-lane mesh cursor / while-while traversal as intersect(), with its state in a struct so a lane can stop
// between steps (other lanes shade) and resume.  Same visit order, same counters, same result.
// ---------------------------------------------------------------------------------------------------
struct Trav {
    f3 lo, ld;             // ray in the current mesh's local space (1/ld is recomputed per round, trav_step)
    float best_t, best_u, best_v, sph_t;
    uint32_t best_tri;     // triangle | orientation<0 << 31, HG_NONE: no mesh hit yet
    uint32_t best_mesh, sph, node, sp, mi;  // mi == n_meshes: traversal finished
    uint64_t live;         // exact-cull mask of the meshes
};

template <bool kMeshLds = false>
__device__ __forceinline__ void trav_begin(const HgKernelParams& kp, const Ray& ray, Trav& t, Counters& c) {
    c.rays++;
    t.sph_t = HG_INF;
    t.sph = isect_spheres(kp, ray, t.sph_t);
    t.best_t = t.sph_t;  // closestIntersection.rayT starts at the sphere hit (:381)
    t.best_u = 0.0f;
    t.best_v = 0.0f;
    t.best_tri = HG_NONE;
    t.best_mesh = 0;
    uint32_t culled = 0;
    const f3 winv = mk(rcp_exact(ray.d.x), rcp_exact(ray.d.y), rcp_exact(ray.d.z));
    t.live = mesh_live_mask(kp, ray.o, winv, t.best_t, culled);
    c.aabb += 2 * culled;
    t.sp = 0;
    t.node = HG_NONE;
    const uint32_t nm = uint32_t(kp.n_meshes);
    t.mi = next_live_mesh(t.live, 0u, nm);
    f3 inv;
    if (t.mi < nm) mesh_local_ray<kMeshLds>(kp, ray, t.mi, t.lo, t.ld, inv, t.node);
}

// One while-while round for the lanes with `act`: descend until each is at a leaf (or out of nodes), test that
// leaf, and move to the next live mesh when the current one is exhausted.
template <bool kMeshLds = false, class Stk>
__device__ __forceinline__ void trav_step(const HgKernelParams& kp, const Ray& ray, Trav& t, Counters& c,
                                          const Stk& stk, bool act, const LeafShare& ls) {
    // 1/ld (the same rcp_exact values mesh_local_ray computes) is not kept in Trav: live only during this round, it
    // stays out of the registers held across the streaming kernel's shading code
    const f3 inv = mk(rcp_exact(t.ld.x), rcp_exact(t.ld.y), rcp_exact(t.ld.z));
    const uint64_t act_mask = wave_ballot(act);  // act is fixed for the round
    const uint32_t dt = kp.descent_t;
    // lanes at an inner node (HG_NONE has the leaf bit): the wave descends while more than dt of them are left, or
    // while every active lane is still descending (relaxed while-while, as in isect_meshes)
    uint64_t dm = act_mask & wave_ballot(int32_t(t.node) >= 0);
    while (dm != 0ull && (uint32_t(__builtin_popcountll(dm)) > dt || dm == act_mask)) {
        c.node_rounds += wave_once();
        if (act && int32_t(t.node) >= 0) {
            const NodePair np = node_pair(kp, t.node);
            const uint32_t refA = pair_ref_a(np), refB = pair_ref_b(np);
            float dA, dB;
            pair_dist(np, t.lo, inv, dA, dB);
            c.aabb += 2;
            const bool bFirst = dB < dA;  // :430-444
            const uint32_t nearRef = bFirst ? refB : refA, farRef = bFirst ? refA : refB;
            const bool nearOk = (bFirst ? dB : dA) < t.best_t, farOk = (bFirst ? dA : dB) < t.best_t;
            if (nearOk && farOk) stk.push(t.sp, farRef);
            t.node = nearOk ? nearRef : farRef;
            if (!nearOk && !farOk) t.node = t.sp > 0 ? stk.pop(t.sp) : HG_NONE;
        }
        dm = act_mask & wave_ballot(int32_t(t.node) >= 0);
    }
    // Distributed leaf test (HG_LEAF_DIST of rounds 1-4: C3 2013 -> 2074 Mpaths/s, leaf-loop lane utilisation 25 % ->
    // 70 %, tools/sweeps/sweep52.txt); check builds fall back to the lane's own sequential loop under a partial EXEC
    const bool at_leaf = act && t.node != HG_NONE && (t.node & HG_LEAF_BIT);
    uint32_t first = 0u, n = 0u;
    if (at_leaf) {
        const uint2 lr = leaf_range(kp, t.node);
        first = lr.x;
        n = lr.y;
    }
    if (leaf_dist(kp, LeafRay{t.lo, t.ld, t.best_t, t.best_u, t.best_v, t.best_tri, t.best_mesh, t.mi}, c, ls, first,
                  n)) {
        if (at_leaf) t.node = t.sp > 0 ? stk.pop(t.sp) : HG_NONE;
    } else if (at_leaf) {  // (HG_CHECK_EXEC builds only) :404-420, the next triangle's loads out before this one's test
        const uint2 leaf = leaf_range(kp, t.node);
        const uint32_t end = leaf.x + leaf.y;
        float4 na, nb;
        float nc;
        tri_load(kp, leaf.x, na, nb, nc);
        for (uint32_t ti = leaf.x; ti < end; ++ti) {
            c.tri_rounds += wave_once();
            const float4 a = na, b = nb;
            const float cz = nc;
            const uint32_t tn = ti + 1 < end ? ti + 1 : ti;
            tri_load(kp, tn, na, nb, nc);
            c.tri++;
            float tt, U, V;
            bool front;
            if (tri_accept(t.lo, t.ld, a, b, cz, t.best_t, tt, U, V, front)) {
                t.best_t = tt;
                t.best_u = U;
                t.best_v = V;
                t.best_tri = ti | (front ? 0u : 0x80000000u);
                t.best_mesh = t.mi;
            }
        }
        t.node = t.sp > 0 ? stk.pop(t.sp) : HG_NONE;
    }
    if (act && t.node == HG_NONE) {
        const uint32_t nm = uint32_t(kp.n_meshes);
        t.mi = next_live_mesh(t.live, t.mi + 1u, nm);
        f3 inv_next;
        if (t.mi < nm) mesh_local_ray<kMeshLds>(kp, ray, t.mi, t.lo, t.ld, inv_next, t.node);
    }
}

// The hit get_ray_intersection returns, from a finished traversal (:452-471 and the sphere pass).
template <bool kMeshLds = false>
__device__ __forceinline__ Hit trav_hit(const HgKernelParams& kp, const Ray& ray, const Trav& t) {
    Hit h;
    h.t = t.sph_t;
    h.orient = 0.0f;
    h.pos = mk(0, 0, 0);
    h.n = mk(0, 0, 0);
    h.mat = 0;
    if (t.best_t < (t.sph_t - 0.0001f) && t.best_t < kp.far_)
        resolve_mesh<kMeshLds>(kp, ray, t.best_t, t.best_u, t.best_v, t.best_tri, t.best_mesh, h);
    else if (t.sph != HG_NONE)
        resolve_sphere(kp, ray, t.sph, h);
    return h;
}

// ---------------------------------------------------------------------------------------------------
// Sky (:196-204): TextureCube.SampleLevel (HC:201) with an integral level = bilinear within one mip, seamless across
// faces as D3D10+ filters cube maps (resting_place_4k.exr.meta:32 imports it seamless): a footprint texel beyond a
// face edge is read from the adjacent face, and at a cube corner the missing fourth texel is the average of the
// three that exist.  The same integer adjacency and operation order as the oracle (oracle/hg_oracle.c).
// ---------------------------------------------------------------------------------------------------
// face frames: major axis M, s axis S, t axis T (sc = dot(d, S), tc = dot(d, T)); faces +X,-X,+Y,-Y,+Z,-Z
__device__ __forceinline__ int cube_axis(int tab, int f, int k) {
    constexpr signed char kM[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
    constexpr signed char kS[6][3] = {{0, 0, -1}, {0, 0, 1}, {1, 0, 0}, {1, 0, 0}, {1, 0, 0}, {-1, 0, 0}};
    constexpr signed char kT[6][3] = {{0, -1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}, {0, -1, 0}, {0, -1, 0}};
    return tab == 0 ? kM[f][k] : tab == 1 ? kS[f][k] : kT[f][k];
}
// texel (i, j) one step off face f -> the adjacent face's texel (exact integer form, see the oracle's cube_adjacent)
__device__ __forceinline__ void cube_adjacent(int f, int i, int j, int size, int& nf, int& ni, int& nj) {
    const int a = 2 * i + 1 - size, b = 2 * j + 1 - size;
    int P[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) P[k] = size * cube_axis(0, f, k) + a * cube_axis(1, f, k) + b * cube_axis(2, f, k);
    int g = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (P[k] == size + 1 || P[k] == -(size + 1)) g = 2 * k + (P[k] < 0 ? 1 : 0);
    int c[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int v = P[0] * cube_axis(1 + e, g, 0) + P[1] * cube_axis(1 + e, g, 1) + P[2] * cube_axis(1 + e, g, 2);
        c[e] = (v == size || v == -size) ? (v > 0 ? size - 1 : 0) : (v + size - 1) / 2;
    }
    nf = g;
    ni = c[0];
    nj = c[1];
}
__device__ f3 sample_sky(const HgKernelParams& kp, f3 dir, int level) {
    if (!(kp.use_cube > 0)) return mk(0, 0, 0);
    float x = dir.x, y = dir.y, z = dir.z;
    float ax = fabsf(x), ay = fabsf(y), az = fabsf(z);
    int face;
    float sc, tc, ma;
    if (az >= ax && az >= ay) {
        ma = az;
        if (z >= 0) { face = 4; sc = x; tc = -y; } else { face = 5; sc = -x; tc = -y; }
    } else if (ay >= ax) {
        ma = ay;
        if (y >= 0) { face = 2; sc = x; tc = z; } else { face = 3; sc = x; tc = -z; }
    } else {
        ma = ax;
        if (x >= 0) { face = 0; sc = -z; tc = -y; } else { face = 1; sc = z; tc = -y; }
    }
    level = level < 0 ? 0 : (level > kp.cube_mips - 1 ? kp.cube_mips - 1 : level);
    int size = kp.cube_size >> level;
    size = size < 1 ? 1 : size;
    const float4* mip = kp.cube + kp.cube_mip_offset[level];
    float s = (sc / ma + 1.0f) * 0.5f;
    float t = (tc / ma + 1.0f) * 0.5f;
    float u = s * float(size) - 0.5f, v = t * float(size) - 0.5f;
    float fu = floorf(u), fv = floorf(v);
    float fx = u - fu, fy = v - fv;
    const int x0 = int(fu), y0 = int(fv);
    f3 tex[2][2];  // [row][col]
    int corner = -1;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int i = x0 + q, j = y0 + r;
            const bool in_i = i >= 0 && i < size, in_j = j >= 0 && j < size;
            tex[r][q] = mk(0, 0, 0);
            if (!in_i && !in_j) {
                corner = r * 2 + q;
                continue;
            }
            int f = face, ii = i, jj = j;
            if (!in_i || !in_j) cube_adjacent(face, i, j, size, f, ii, jj);
            tex[r][q] = xyz(mip[(size_t(f) * size + jj) * size + ii]);
        }
    }
    if (corner >= 0) {  // the average of the other three: same row, same column, diagonal
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k != corner) continue;
            const int r = k >> 1, q = k & 1;
            const f3 sum = (tex[r][1 - q] + tex[1 - r][q]) + tex[1 - r][1 - q];
            tex[r][q] = mk(sum.x / 3.0f, sum.y / 3.0f, sum.z / 3.0f);
        }
    }
    const float gx = 1.0f - fx, gy = 1.0f - fy;
    f3 top = tex[0][0] * gx + tex[0][1] * fx;
    f3 bot = tex[1][0] * gx + tex[1][1] * fx;
    return top * gy + bot * fy;
}

__device__ __forceinline__ int sky_level(const HgKernelParams& kp, float acc_rough) {
    float lf = hg_roundf(float(kp.default_mip) + acc_rough * 8.0f);
    if (!(lf >= 0.0f)) return 0;
    if (lf > 64.0f) return 64;
    return int(lf);
}

// ---------------------------------------------------------------------------------------------------
// BSDF (:491-741) and medium stack (:582-665)
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ f3 lambert(f3 n, f3 rv) {  // :491-501
    f3 p = rv + n;
    if (len(p) < 1e-8f) p = n;
    return normalize(p);
}
__device__ __forceinline__ f3 reflect(f3 i, f3 n) { return i - n * (2.0f * dot(i, n)); }  // :506-509

__device__ __forceinline__ float schlick_adjusted(float n1, float n2, f3 nrm, f3 inc, float mn, float mx) {
    float r0 = (n1 - n2) / (n1 + n2);  // :519-540
    r0 *= r0;
    float cosX = -dot(nrm, inc);
    if (n1 > n2) {
        float n = n1 / n2;
        float sinT2 = n * n * (1.0f - cosX * cosX);
        if (sinT2 > 1.0f) return mx;
        cosX = __builtin_sqrtf(1.0f - sinT2);
    }
    float x = 1.0f - cosX;
    float ret = r0 + (1.0f - r0) * x * x * x * x * x;
    return mn + ret * (mx - mn);
}

__device__ __forceinline__ f3 refract_tir(f3 inc, f3 nrm, float n1, float n2, bool& tir) {  // :557-572
    float ct = fminf(dot(-inc, nrm), 1.0f);
    float st = __builtin_sqrtf(1.0f - ct * ct);
    float n12 = n1 / n2;
    if (n12 * st > 1.0f) {
        tir = true;
        return reflect(inc, nrm);
    }
    f3 perp = (inc + nrm * ct) * n12;
    float lp = len(perp);
    f3 par = nrm * (-__builtin_sqrtf(fabsf(1.0f - lp * lp)));
    return perp + par;
}

struct Medium {
    float ior;
    f3 absorb;
    uint32_t id;
};
__device__ __forceinline__ Medium medium_of(const HgKernelParams& kp, uint32_t m) {
    const float4 ai = kp.materials[5 * m + 3];
    const float4 pr = kp.materials[5 * m + 4];
    return Medium{ai.w, xyz(ai), __float_as_uint(pr.y)};
}
__device__ __forceinline__ Medium empty_medium() { return Medium{1.0f, mk(0, 0, 0), 0xFFFFFFFFu}; }
__device__ __forceinline__ Medium top_medium(const HgKernelParams& kp, const MediumStack& ms) {
    return ms.sp > 0 ? medium_of(kp, ms.get(ms.sp - 1)) : empty_medium();
}
__device__ void medium_push(const HgKernelParams& kp, MediumStack& ms, uint32_t m) {  // :582-622
    if (ms.sp == 0) {
        ms.s = uint64_t(m);
        ms.sp = 1;
        return;
    }
    const int32_t prio = mat_priority(kp, m);
    int ins = ms.sp;
    if (prio > mat_priority(kp, ms.get(ms.sp - 1))) {
        for (int i = ms.sp - 1; i >= 0; --i) {
            if (prio < mat_priority(kp, ms.get(i))) {
                ins = i + 1;
                break;
            }
        }
        if (ins == ms.sp) ins = 0;
    }
    if (ms.sp >= 8) return;  // overflow: dropped (reference UB; same rule in the oracle)
    const uint64_t low_mask = ins == 0 ? 0ull : (~0ull >> (64 - 8 * ins));
    const uint64_t low = ms.s & low_mask;
    const uint64_t high = ms.s & ~low_mask;
    ms.s = low | (high << 8) | (uint64_t(m) << (8 * ins));
    ms.sp++;
}
__device__ void medium_pop(const HgKernelParams& kp, MediumStack& ms, uint32_t id) {  // :627-642
    for (int i = 0; i < ms.sp; ++i) {
        if (medium_of(kp, ms.get(i)).id == id) {
            const uint64_t low_mask = i == 0 ? 0ull : (~0ull >> (64 - 8 * i));
            const uint64_t low = ms.s & low_mask;
            const uint64_t high = (i + 1 < 8) ? ((ms.s >> (8 * (i + 1))) << (8 * i)) : 0ull;
            ms.s = low | high;
            ms.sp--;
            return;
        }
    }
}

// material_BRDF :672-741
__device__ f3 material_brdf(const HgKernelParams& kp, const Sampler& smp, Ray& ray, const Hit& hit, const Mat& mt,
                            const Medium& cur, const Medium& hm, uint32_t& bt) {
    f3 att;
    float rr0, rr1, pr0, pr1;
    smp.get2(ID_ROUGH, rr0, rr1);
    smp.get2(ID_PROPERTY, pr0, pr1);
    // get_random_unit_vector (HalogenRandom.hlsl:282-298)
    const float theta = rr0 * 2.0f * HLSL_PI;
    const float phi = hg_acosf_fused(2.0f * rr1 - 1.0f);  // = hg_acosf (tests/test_fmath.py, every input)
    float sT, cT, sP, cP;  // = hg_sinf / hg_cosf of each angle, one reduction per angle (tests/test_fmath.py)
    hg_sincosf(theta, &sT, &cT);
    hg_sincosf(phi, &sP, &cP);
    const f3 rv = mk(1.0f * sP * cT, 1.0f * sP * sT, 1.0f * cP);
    const float rough2 = mt.prio_id_r2.z;
    if (!(pr0 > mt.albedo.w)) {
        att = xyz(mt.albedo);
        const f3 diffuse = lambert(hit.n, rv);
        const float metallic = mt.spec_metal.w;
        const float thr = (metallic > 0.0f) ? schlick_adjusted(cur.ior, hm.ior, hit.n, ray.d, metallic, 1.0f)
                                            : metallic;
        const bool spec = pr1 < thr;
        bt = spec ? 1u : 0u;
        if (spec) {
            ray.d = lerp(reflect(ray.d, hit.n), diffuse, rough2);
            att = xyz(mt.spec_metal);
        } else {
            ray.d = diffuse;
        }
        ray.o = hit.pos + hit.n * 0.0001f;
    } else {
        bt = 2u;
        att = mk(1, 1, 1);
        bool tir = false;
        ray.d = refract_tir(ray.d, hit.n, cur.ior, hm.ior, tir);
        const f3 dd = tir ? lambert(hit.n, rv) : lambert(-hit.n, rv);
        ray.d = lerp(ray.d, dd, rough2);
        ray.o = hit.pos - hit.n * 0.0001f;
    }
    ray.d = normalize(ray.d);
    return att;
}

// evaluate_material_hit :743-817
// bt_out: the bounceTypes[] slot this hit increments (0 diffuse, 1 glossy, 2 transmission; a false hit counts as
// transmission, :806)
__device__ f3 evaluate_hit(const HgKernelParams& kp, const Sampler& smp, MediumStack& ms, Ray& ray, const Hit& hit,
                           const Mat& mt, uint32_t& bt_out) {
    const Medium internal = medium_of(kp, hit.mat);
    const int32_t prio = __float_as_int(mt.prio_id_r2.x);
    Medium cur, hm;
    bool trueHit = true;
    if (prio >= 0) {
        trueHit = ms.sp == 0 || prio <= mat_priority(kp, ms.get(ms.sp - 1));
        if (hit.orient == 1.0f) {
            cur = top_medium(kp, ms);
            hm = internal;
            medium_push(kp, ms, hit.mat);
        } else {
            cur = ms.sp == 0 ? internal : top_medium(kp, ms);
            medium_pop(kp, ms, internal.id);
            hm = top_medium(kp, ms);
        }
    } else {
        if (hit.orient == 1.0f) {
            cur = top_medium(kp, ms);
            hm = internal;
        } else {
            cur = internal;
            hm = top_medium(kp, ms);
        }
    }
    f3 att;
    if (trueHit) {
        uint32_t bt = 0;
        att = material_brdf(kp, smp, ray, hit, mt, cur, hm, bt);
        bt_out = bt;
        if (hit.orient > 0.0f && bt != 2u) medium_pop(kp, ms, internal.id);
    } else {
        ray.o = hit.pos - hit.n * 0.0001f;
        att = mk(1, 1, 1);
        bt_out = 2u;
    }
    if (cur.id != 0xFFFFFFFFu) {
        att = mk(att.x * hg_expf(-cur.absorb.x * hit.t), att.y * hg_expf(-cur.absorb.y * hit.t),
                 att.z * hg_expf(-cur.absorb.z * hit.t));
    }
    return att;
}

// trace_ray :876-950
template <class Stk>
__device__ f3 trace_ray(const HgKernelParams& kp, Sampler& smp, MediumStack& ms, Ray ray, Counters& c,
                        const Stk& stk) {
    f3 acc = mk(0, 0, 0), thr = mk(1, 1, 1);
    float acc_rough = 0.0f;
    Bounces bounce{0, 0, 0};
    for (uint32_t it = 0; it <= kp.max_bounces; ++it) {
        if (bounce.diffuse > kp.max_diff || bounce.glossy > kp.max_glossy || bounce.transmission > kp.max_trans)
            break;
        const Hit hit = intersect(kp, ray, c, stk);
        if (hit.t < kp.far_) {
            c.hits++;
            const Mat mt = load_mat(kp, hit.mat);
            acc = acc + xyz(mt.emis_rough) * thr;
            uint32_t bt = 0;
            const f3 att = evaluate_hit(kp, smp, ms, ray, hit, mt, bt);
            bounce.bump(bt);
            thr = thr * att;
            acc_rough += mt.emis_rough.w * thr.x;  // float3 -> float truncation (:911)
            const float rr = smp.get1(ID_RR);
            smp.offset += BOUNCE_INC;
            const float contribution = fmaxf(fmaxf(thr.x, thr.y), thr.z);
            if (rr > contribution) break;
            thr = thr * rcp_exact(contribution);
        } else {
            c.primary_miss += it == 0u;
            acc = acc + sample_sky(kp, ray.d, sky_level(kp, acc_rough)) * thr;
            break;
        }
    }
    return acc;
}

// trace_ray_debug :952-982
template <class Stk>
__device__ f3 trace_ray_debug(const HgKernelParams& kp, Sampler& smp, MediumStack& ms, Ray ray, Counters& c,
                              const Stk& stk) {
    const uint32_t tri0 = c.tri, box0 = c.aabb;  // TriangleTests = AABBTests = 0
    switch (kp.debug_mode) {
        default:
            return mk(0, 0, 0);
        case 1: {
            const Hit h = intersect(kp, ray, c, stk);
            if (h.t < kp.far_) return xyz(kp.materials[5 * h.mat]);
            return sample_sky(kp, ray.d, kp.default_mip);
        }
        case 2: {
            const Hit h = intersect(kp, ray, c, stk);
            if (h.t < kp.far_) return mk((h.n.x + 1.0f) / 2.0f, (h.n.y + 1.0f) / 2.0f, (h.n.z + 1.0f) / 2.0f);
            return sample_sky(kp, ray.d, kp.default_mip);
        }
        case 3:
        case 4:
        case 5: {
            trace_ray(kp, smp, ms, ray, c, stk);
            const uint32_t tt = c.tri - tri0, bb = c.aabb - box0;
            if (kp.debug_mode == 3) {
                if (tt > kp.tri_range) return mk(1, 1, 1);
                return mk(float(tt) / float(kp.tri_range), 0, 0);
            }
            if (kp.debug_mode == 4) {
                if (bb > kp.box_range) return mk(1, 1, 1);
                return mk(float(bb) / float(kp.box_range), 0, 0);
            }
            if (tt > kp.tri_range || bb > kp.box_range) return mk(1, 1, 1);
            return mk(float(tt) / float(kp.tri_range), 0, float(bb) / float(kp.box_range));
        }
    }
}

// inverted_blackman_harris_cdf_approximation (HalogenRandom.hlsl:319-330)
__device__ __forceinline__ float inv_blackman_harris(float x) {
    const float a = (x * 1.99221575606f) - 0.99610787803f;
    return (0.5f * hg_logf((1.0f + a) / (1.0f - a))) / 6.24f;
}

// get_ray :996-1013 (+ get_ray_jitter :984-994, get_random_point_circle HalogenRandom.hlsl:303-308)
__device__ Ray camera_ray(const HgKernelParams& kp, const Sampler& smp, float ndcx, float ndcy) {
    float j0, j1;
    f3 ap = mk(0.0f, 0.0f, 0.0f);
    // Pinhole (disc radius 0): ap is (+-0, +-0, 0), the zeros' signs those of cos / sin.  Nothing below can see them
    // when the camera translation has no zero component (m[3] + (+-0) = m[3] in xform) and pf has no -0 component:
    // ndcx, ndcy are never -0 (x - 1 rounds an exact 0 to +0), so with vw, vh > 0 screen.x, .y are never -0 either
    // (+0 + -0 = +0; no sum underflows), and normalize / the focal distance > 0 keep the sign.  Then pf - (+-0) = pf,
    // and the focal sample and its sincos are skipped: the same bits.
    if (!(kp.focal_disc_radius == 0.0f && kp.cam[3] != 0.0f && kp.cam[7] != 0.0f && kp.cam[11] != 0.0f &&
          kp.vw > 0.0f && kp.vh > 0.0f && kp.near_ > 0.0f && kp.focal_dist > 0.0f)) {
        float fd0, fd1;
        smp.get2(ID_FOCAL, fd0, fd1);
        const float th = (fd0 * 360.0f) * HG_DEG2RAD;
        float sth, cth;
        hg_sincosf(th, &sth, &cth);
        ap = mk(cth * kp.focal_disc_radius * fd1, sth * kp.focal_disc_radius * fd1, 0.0f);
    }
    f3 screen = mk(ndcx * kp.vw, ndcy * kp.vh, 1.0f * kp.near_);
    smp.get2(ID_JITTER, j0, j1);
    const float jx = (inv_blackman_harris(j0) - 0.5f) * 2.0f * kp.filter_radius * kp.psx;
    const float jy = (inv_blackman_harris(j1) - 0.5f) * 2.0f * kp.filter_radius * kp.psy;
    screen = screen + mk(jx, jy, 0.0f);
    const f3 pf = normalize(screen) * kp.focal_dist;
    const f3 csd = normalize(pf - ap);
    Ray r;
    r.o = xform(kp.cam, ap, 1.0f);
    r.d = normalize(xform(kp.cam, csd, 0.0f));
    return r;
}

// wave64 sum (all 64 lanes active at the call site)
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace hgd

