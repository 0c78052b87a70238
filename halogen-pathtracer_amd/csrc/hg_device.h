// hg_device.h — device-side building blocks of the Halogen hot path shared by the kernels
// (hg_mega.hip: one-thread-per-pixel megakernel; hg_wavefront.hip: regenerating wavefront pipeline).
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
// normalize = v * (1/sqrt(dot(v,v))) (hg_fmath.h hg_rnorm) with the correctly rounded reciprocal (same bits)
#if HG_RCP_NORMALIZE
__device__ __forceinline__ f3 normalize(f3 a) { return a * rcp_exact(__builtin_sqrtf(dot(a, a))); }
#else
__device__ __forceinline__ f3 normalize(f3 a) { return a * hg_rnorm(dot(a, a)); }
#endif
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

// XCD-aware block order: the dispatcher deals workgroups round-robin to the 8 XCDs (b % 8), each with its own
// L2.  Remapping b -> a contiguous range per XCD gives every XCD its own band of tiles, so the BVH nodes its
// waves touch overlap more in its L2.  A bijection on [0, n) whatever the real placement (speed only).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t n) {
#if HG_XCD_REMAP
    const uint32_t xcd = b & 7u, k = b >> 3, per = n >> 3, rem = n & 7u;
    return xcd < rem ? xcd * (per + 1u) + k : rem * (per + 1u) + (xcd - rem) * per + k;
#else
    (void)n;
    return b;
#endif
}

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
// HG_PHASE_DETAIL analysis builds: add the wave clock elapsed since `since` to counter slot `slot` (from the first
// active lane, so it works inside divergent code) and return the new clock.
__device__ __forceinline__ uint64_t phase_mark(const HgKernelParams& kp, int slot, uint64_t since) {
    const uint64_t t = wave_clock();
    if (int(threadIdx.x & 63u) == __ffsll((unsigned long long)__ballot(1)) - 1)
        atomicAdd(kp.counters + slot, (unsigned long long)(t - since));
    return wave_clock();
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
#if HG_MAT_SCALAR
    // every active lane shading the same material (one glass, one wall): five scalar loads through the constant
    // cache instead of five vector-memory instructions on the texture-data unit that binds the kernel
    const uint32_t m0 = uint32_t(__builtin_amdgcn_readfirstlane(int(m)));
    if (__builtin_amdgcn_ballot_w64(m != m0) == 0ull) {
        typedef const __attribute__((address_space(4))) float* cfp;
        const cfp q = (cfp)(uintptr_t)(kp.materials + 5u * m0);
        return Mat{make_float4(q[0], q[1], q[2], q[3]), make_float4(q[4], q[5], q[6], q[7]),
                   make_float4(q[8], q[9], q[10], q[11]), make_float4(q[12], q[13], q[14], q[15]),
                   make_float4(q[16], q[17], q[18], q[19])};
    }
#endif
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

// Frame colour of launch frame f (0 .. n_frames-1) for accumulator slot `slot` (hg_blend_frames reads the same layout)
__device__ __forceinline__ size_t fc_slot_frame(size_t slot, uint32_t f, size_t n_slots, uint32_t n_frames) {
#if HG_FC_SLOT_MAJOR
    (void)n_slots;
    return slot * size_t(n_frames) + f;
#else
    (void)n_frames;
    return size_t(f) * n_slots + slot;
#endif
}
// Frame colours are written once by the trace and read once by the blend: with HG_FC_NT both go through the
// non-temporal hint, so the 2.1 GB a 64-frame C3 launch writes is not kept in L2 ahead of the BVH lines
__device__ __forceinline__ void fc_store(float4* p, float4 v) {
#if HG_FC_NT
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z);
    __builtin_nontemporal_store(v.w, &p->w);
#else
    *p = v;
#endif
}
__device__ __forceinline__ float4 fc_load(const float4* p) {
#if HG_FC_NT
    return make_float4(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y),
                       __builtin_nontemporal_load(&p->z), __builtin_nontemporal_load(&p->w));
#else
    return *p;
#endif
}
__device__ __forceinline__ size_t fc_index(const HgKernelParams& kp, uint32_t f, size_t slot) {
    return fc_slot_frame(slot, f, size_t(uint32_t(kp.n_local_tiles)) * 64u, uint32_t(kp.n_frames));
}

// Triangle ti's Moller-Trumbore operands from the three SoA streams: a = (v0, e1.x), b = (e1.yz, e2.xy), cz = e2.z.
// (One 48-B record per triangle instead was measured: C3 -0.3 %, C2 -5.7 %, C5 -2.4 %, tools/sweeps/NOTES_r02.md;
// the non-temporal hint on these loads: C3 -9.7 %, C3F -10 %, tools/sweeps/sweep_r03_o.jsonl.)
__device__ __forceinline__ void tri_load(const HgKernelParams& kp, uint32_t ti, float4& a, float4& b, float& cz) {
#if HG_TRI_AOS
    typedef float hg_v4u __attribute__((ext_vector_type(4), aligned(4)));  // 4-B aligned 16-B loads
    const char* p = reinterpret_cast<const char*>(kp.tri_a) + ti * 36u;
    const hg_v4u va = *reinterpret_cast<const hg_v4u*>(p), vb = *reinterpret_cast<const hg_v4u*>(p + 16);
    a = make_float4(va.x, va.y, va.z, va.w);
    b = make_float4(vb.x, vb.y, vb.z, vb.w);
    cz = *reinterpret_cast<const float*>(p + 32);
#else
    a = ld_off(kp.tri_a, ti << 4);
    b = ld_off(kp.tri_b, ti << 4);
    cz = ld_off(kp.tri_c, ti << 2);
#endif
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

// A child-pair record (hg_runtime.hip, BLAS pass 2): both children's boxes and refs in 64 B, 56 of them used.
// HG_PAIR_SOA lays the boxes out coordinate by coordinate with A and B side by side, so that the two box tests of a
// descent step run on packed FP32 pairs (v_pk_add_f32 / v_pk_mul_f32: two IEEE operations per instruction, the same
// results as the scalar ones):
//   q0 = (A.lo.x, B.lo.x, A.lo.y, B.lo.y), q1 = (A.lo.z, B.lo.z, A.hi.x, B.hi.x), q2 = (A.hi.y, B.hi.y, A.hi.z, B.hi.z),
//   q3 = (refA, refB, -, -);
// otherwise q0 = (A.lo, refA), q1 = (A.hi, refB), q2 = (B.lo, -), q3 = (B.hi, -).
struct NodePair {
    float4 q0, q1, q2, q3;
};
__device__ __forceinline__ NodePair node_pair(const HgKernelParams& kp, uint32_t node) {
    const uint32_t ro = node << 6;
#if HG_PAIR_SOA
    const uint2 refs = ld_off(reinterpret_cast<const uint2*>(kp.nodes), ro + 48);
    return NodePair{ld_off(kp.nodes, ro), ld_off(kp.nodes, ro + 16), ld_off(kp.nodes, ro + 32),
                    make_float4(__uint_as_float(refs.x), __uint_as_float(refs.y), 0.0f, 0.0f)};
#else
    return NodePair{ld_off(kp.nodes, ro), ld_off(kp.nodes, ro + 16), ld_off(kp.nodes, ro + 32), ld_off(kp.nodes, ro + 48)};
#endif
}
__device__ __forceinline__ NodePair node_pair_at(const float4* p) { return NodePair{p[0], p[1], p[2], p[3]}; }
__device__ __forceinline__ uint32_t pair_ref_a(const NodePair& r) {
    return __float_as_uint(HG_PAIR_SOA ? r.q3.x : r.q0.w);
}
__device__ __forceinline__ uint32_t pair_ref_b(const NodePair& r) {
    return __float_as_uint(HG_PAIR_SOA ? r.q3.y : r.q1.w);
}
// ray_aabb (:244-259) of both children: dA, dB
__device__ __forceinline__ void pair_dist(const NodePair& r, f3 o, f3 inv, float& dA, float& dB) {
#if HG_PAIR_SOA
    typedef float v2f __attribute__((ext_vector_type(2)));
    const v2f lx = (v2f{r.q0.x, r.q0.y} - o.x) * inv.x, ly = (v2f{r.q0.z, r.q0.w} - o.y) * inv.y;
    const v2f lz = (v2f{r.q1.x, r.q1.y} - o.z) * inv.z, hx = (v2f{r.q1.z, r.q1.w} - o.x) * inv.x;
    const v2f hy = (v2f{r.q2.x, r.q2.y} - o.y) * inv.y, hz = (v2f{r.q2.z, r.q2.w} - o.z) * inv.z;
    float aMin = fminf(lx.x, hx.x), aMax = fmaxf(lx.x, hx.x);
    aMin = fmaxf(aMin, fminf(ly.x, hy.x));
    aMax = fminf(aMax, fmaxf(ly.x, hy.x));
    aMin = fmaxf(aMin, fminf(lz.x, hz.x));
    aMax = fminf(aMax, fmaxf(lz.x, hz.x));
    float bMin = fminf(lx.y, hx.y), bMax = fmaxf(lx.y, hx.y);
    bMin = fmaxf(bMin, fminf(ly.y, hy.y));
    bMax = fminf(bMax, fmaxf(ly.y, hy.y));
    bMin = fmaxf(bMin, fminf(lz.y, hz.y));
    bMax = fminf(bMax, fmaxf(lz.y, hz.y));
    dA = aMax > fmaxf(0.0f, aMin) ? aMin : HG_INF;
    dB = bMax > fmaxf(0.0f, bMin) ? bMin : HG_INF;
#else
    dA = ray_aabb(xyz(r.q0), xyz(r.q1), o, inv);
    dB = ray_aabb(xyz(r.q2), xyz(r.q3), o, inv);
#endif
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
// The mesh loop is wave-uniform (mesh records come through the scalar cache); inside a mesh the traversal keeps
// the current node in a register (the reference's push-near-then-pop-near is a no-op on order) and runs
// while-while: all lanes descend inner nodes together until each holds a leaf, then test one leaf each.
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
#if HG_LANE_MESHES
    // Per-lane mesh cursor: each lane walks its own live meshes in buffer order (the reference's order, so ties
    // resolve identically) and moves to its next mesh as soon as it finishes one, so a wave waits for the lane
    // with the most total work instead of the slowest lane of every mesh in turn.
    const uint32_t nm = uint32_t(kp.n_meshes);
    uint32_t mi = next_live_mesh(live, 0u, nm);
    bool active = mi < nm;
    f3 lo = mk(0, 0, 0), ld = mk(0, 0, 0), inv = mk(0, 0, 0);
    uint32_t node = HG_NONE, sp = 0;
    if (active) mesh_local_ray<kMeshLds>(kp, ray, mi, lo, ld, inv, node);
    while (__any(active)) {
#if HG_TRAV_IFIF
        if (active && !(node & HG_LEAF_BIT)) {  // if-if: one node step per round, leaves tested in the same round
#else
        // while-while, relaxed: descend while more than kp.descent_t lanes are still descending (0: until every
        // lane is at a leaf), and in any case until at least one lane can make other progress (a leaf to test or
        // its mesh finished); the few stragglers pause while the others test their leaves.  Each lane's own
        // sequence of node / leaf steps is unchanged.
        const uint64_t act_mask = wave_ballot(active);
        const uint32_t dt = kp.descent_t;
        for (uint64_t dm = act_mask & wave_ballot(int32_t(node) >= 0);
             dm != 0ull && (uint32_t(__builtin_popcountll(dm)) > dt || dm == act_mask);
             dm = act_mask & wave_ballot(int32_t(node) >= 0)) {
            c.node_rounds += wave_once();
            if (active && int32_t(node) >= 0) {
#endif
                const NodePair np = node_pair(kp, node);
                float dA, dB;
                pair_dist(np, lo, inv, dA, dB);
                c.aabb += 2;
                const uint32_t refA = pair_ref_a(np), refB = pair_ref_b(np);
                // reference (:430-444): push far, push near (each only if tEntry < closest), pop near
                const bool bFirst = dB < dA;
                const uint32_t nearRef = bFirst ? refB : refA, farRef = bFirst ? refA : refB;
                const bool nearOk = (bFirst ? dB : dA) < best_t, farOk = (bFirst ? dA : dB) < best_t;
                // near (far pushed if it is also entered), else far, else pop — decided branch-free
#if HG_BRANCHLESS_DESCENT
                if (nearOk && farOk) stk.push(sp, farRef);
                node = nearOk ? nearRef : farRef;
                if (!nearOk && !farOk) node = sp > 0 ? stk.pop(sp) : HG_NONE;
#else
                if (nearOk) {
                    if (farOk) stk.push(sp, farRef);
                    node = nearRef;
                } else if (farOk) {
                    node = farRef;
                } else {
                    node = sp > 0 ? stk.pop(sp) : HG_NONE;
                }
#endif
#if HG_TRAV_IFIF
        } else
#else
            }
        }
#endif
        if (active && node != HG_NONE && (node & HG_LEAF_BIT)) {  // a leaf: its triangles in order (:404-420)
            const uint2 leaf = leaf_range(kp, node);
            const uint32_t end = leaf.x + leaf.y;
#if HG_TRI_PREFETCH
            float4 na, nb;
            float nc;
            tri_load(kp, leaf.x, na, nb, nc);
#endif
            for (uint32_t ti = leaf.x; ti < end; ++ti) {
                c.tri_rounds += wave_once();
#if HG_TRI_PREFETCH  // the next triangle's loads go out before this one is tested
                const float4 a = na, b = nb;
                const float cz = nc;
                const uint32_t tn = ti + 1 < end ? ti + 1 : ti;
                tri_load(kp, tn, na, nb, nc);
#else
                float4 a, b;
                float cz;
                tri_load(kp, ti, a, b, cz);
#endif
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
#else
    for (int mi = 0; mi < kp.n_meshes; ++mi) {
        bool active = mi >= 64 || ((live >> mi) & 1ull);
        if (!__any(active)) continue;  // the whole wave skips this mesh
        if (!active) continue;
        const float4* md4 = reinterpret_cast<const float4*>(kp.meshes + mi);
        const float4 c0 = md4[0], c1 = md4[1], c2 = md4[2], c3 = md4[3];  // worldToLocal columns
        const uint32_t root = __float_as_uint(md4[4].x);
        // world -> local, direction NOT normalized (:390-392)
        const f3 lo = mk(((c0.x * ray.o.x + c1.x * ray.o.y) + c2.x * ray.o.z) + c3.x * 1.0f,
                         ((c0.y * ray.o.x + c1.y * ray.o.y) + c2.y * ray.o.z) + c3.y * 1.0f,
                         ((c0.z * ray.o.x + c1.z * ray.o.y) + c2.z * ray.o.z) + c3.z * 1.0f);
        const f3 ld = mk(((c0.x * ray.d.x + c1.x * ray.d.y) + c2.x * ray.d.z) + c3.x * 0.0f,
                         ((c0.y * ray.d.x + c1.y * ray.d.y) + c2.y * ray.d.z) + c3.y * 0.0f,
                         ((c0.z * ray.d.x + c1.z * ray.d.y) + c2.z * ray.d.z) + c3.z * 0.0f);
        const f3 inv = mk(rcp_exact(ld.x), rcp_exact(ld.y), rcp_exact(ld.z));
        uint32_t node = root, sp = 0;  // root pushed untested (:401), held in a register
        while (__any(active)) {
            while (__any(active && !(node & HG_LEAF_BIT))) {
                if (active && !(node & HG_LEAF_BIT)) {
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
            if (active && node != HG_NONE && (node & HG_LEAF_BIT)) {  // a leaf: its triangles in order
                const uint2 leaf = leaf_range(kp, node);
                uint32_t ti = leaf.x;
                const uint32_t end = leaf.x + leaf.y;
#if HG_TRI_PREFETCH
                float4 ta, tb;
                float tc;
                tri_load(kp, ti, ta, tb, tc);
#endif
                for (; ti < end; ++ti) {
#if HG_TRI_PREFETCH
                    const float4 a = ta, b = tb;
                    const float cz = tc;
                    if (ti + 1 < end) {
                        tri_load(kp, ti + 1, ta, tb, tc);
                    }
#else
                    float4 a, b;
                    float cz;
                    tri_load(kp, ti, a, b, cz);
#endif
                    c.tri++;
                    float t, U, V;
                    bool front;
                    if (tri_accept(lo, ld, a, b, cz, best_t, t, U, V, front)) {
                        best_t = t;
                        best_u = U;
                        best_v = V;
                        best_tri = ti | (front ? 0u : 0x80000000u);
                        best_mesh = uint32_t(mi);
                    }
                }
                node = sp > 0 ? stk.pop(sp) : HG_NONE;
            }
            if (node == HG_NONE) active = false;
        }
    }
#endif
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
#if HG_NODE_PREFETCH
// Prefetch the 128-B line holding the children's records (DFS pair layout: siblings share a line) while the
// current record's boxes are tested: a 4-B load straight into a per-wave LDS sink (no VGPR is written), whose only
// purpose is to pull the line into the caches before the next round asks for it.
__shared__ uint32_t hg_prefetch_sink[64];
__device__ __forceinline__ void node_prefetch(const HgKernelParams& kp, uint32_t refA, uint32_t refB) {
    const uint32_t pf = !(refA & HG_LEAF_BIT) ? refA : refB;
    if (!(pf & HG_LEAF_BIT))
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(uintptr_t)(reinterpret_cast<const char*>(kp.nodes) +
                                                                       (size_t(pf) << 6)),
            (__attribute__((address_space(3))) void*)hg_prefetch_sink, 4, 0, 0);
}
#endif

#if HG_QUAD_FETCH
// Quad-cooperative node fetch (DESIGN.md §10 lever 4).  A descent step loads one 64-B record per lane with four 16-B
// loads, each touching up to 64 records per wave instruction, and the texture data path prices an instruction by the
// lines it touches.  Here the four lanes of each quad load their four records one after another (round j: lane q loads
// quarter q of quad-lane j's record, so an instruction touches at most 16 records, each as one contiguous 64 B), and a
// 4x4 transpose inside the quad (two DPP butterfly stages) hands every lane its own record: the same bytes, the same
// result.  Every lane of the wave must take part (trav_step runs with the whole wave active).
template <int kCtrl>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    return uint32_t(__builtin_amdgcn_mov_dpp(int(v), kCtrl, 0xF, 0xF, true));
}
template <int kCtrl>
__device__ __forceinline__ float qpermf(float v) { return __uint_as_float(qperm<kCtrl>(__float_as_uint(v))); }
// one butterfly stage over columns (a, b) = (j, j ^ s): a' = hi ? partner's b : a, b' = hi ? b : partner's a
template <int kCtrl>
__device__ __forceinline__ void quad_stage(float4& a, float4& b, bool hi) {
    const float4 pa = make_float4(qpermf<kCtrl>(a.x), qpermf<kCtrl>(a.y), qpermf<kCtrl>(a.z), qpermf<kCtrl>(a.w));
    const float4 pb = make_float4(qpermf<kCtrl>(b.x), qpermf<kCtrl>(b.y), qpermf<kCtrl>(b.z), qpermf<kCtrl>(b.w));
    a = make_float4(hi ? pb.x : a.x, hi ? pb.y : a.y, hi ? pb.z : a.z, hi ? pb.w : a.w);
    b = make_float4(hi ? b.x : pa.x, hi ? b.y : pa.y, hi ? b.z : pa.z, hi ? b.w : pa.w);
}
// The records of the lanes with `want` (others: unspecified); false = the caller loads per lane (adaptive mode chose
// the per-lane path for this step)
__device__ __forceinline__ bool quad_node_fetch(const HgKernelParams& kp, bool want, uint32_t node, float4& c0,
                                                float4& c1, float4& c2, float4& c3) {
    const uint32_t q = __lane_id() & 3u;
    const uint32_t key = want ? node : HG_NONE;
    const uint32_t k0 = qperm<0x00>(key), k1 = qperm<0x55>(key), k2 = qperm<0xAA>(key), k3 = qperm<0xFF>(key);
#if HG_QUAD_FETCH == 2
    // quads that need 2+ distinct records (where one full-record load per round beats four 64-record loads)
    const bool spread = q == 0u && ((k1 != k0 && k1 != HG_NONE && k0 != HG_NONE) ||
                                    (k2 != k0 && k2 != k1 && k2 != HG_NONE) ||
                                    (k3 != k0 && k3 != k1 && k3 != k2 && k3 != HG_NONE));
    if (wave_count(spread) < uint32_t(HG_QUAD_MIN)) return false;
#endif
    const uint32_t qo = q << 4;
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, r2 = r0, r3 = r0;
    if (k0 != HG_NONE) r0 = ld_off(kp.nodes, (k0 << 6) + qo);
    if (k1 != HG_NONE) r1 = ld_off(kp.nodes, (k1 << 6) + qo);
    if (k2 != HG_NONE) r2 = ld_off(kp.nodes, (k2 << 6) + qo);
    if (k3 != HG_NONE) r3 = ld_off(kp.nodes, (k3 << 6) + qo);
    // r_j holds quarter q of quad-lane j's record; transpose so that lane q holds quarters 0..3 of its own
    const bool h1 = (q & 1u) != 0u, h2 = (q & 2u) != 0u;
    quad_stage<0xB1>(r0, r1, h1);  // quad_perm 1,0,3,2
    quad_stage<0xB1>(r2, r3, h1);
    quad_stage<0x4E>(r0, r2, h2);  // quad_perm 2,3,0,1
    quad_stage<0x4E>(r1, r3, h2);
    c0 = r0;
    c1 = r1;
    c2 = r2;
    c3 = r3;
    return true;
}
#endif

#if HG_NODE_DEDUP
// Wave-level deduplicated node fetch (DESIGN.md §10 lever 10).  A descent round's loading lanes need few distinct
// records (C3: 5-16 in 48 % of rounds, 17-32 in 47 %, more in 0.07 %; tools/coherence_stats.py), yet each lane
// loading its own 64-B record costs the texture-data unit four wave instructions whatever the sharing.  Here the
// distinct records are enumerated (one readlane + ballot per record), packed densely into lanes (4 lanes x 16 B per
// record when at most 16, else 2 lanes x 2 x 16 B), fetched with one or two wave instructions, and every lane takes
// its record's 16 words from their lanes with ds_bpermute.  The same bytes: the same results.  Returns false (the
// caller loads per lane) when more than 32 records are needed.  The whole wave must be active.
__device__ __forceinline__ uint32_t bperm_u(uint32_t src_lane, uint32_t v) {
    return uint32_t(__builtin_amdgcn_ds_bpermute(int(src_lane << 2), int(v)));
}
__device__ __forceinline__ float4 bperm_f4(uint32_t src_lane, const float4& v) {
    const int a = int(src_lane << 2);
    return make_float4(__int_as_float(__builtin_amdgcn_ds_bpermute(a, __float_as_int(v.x))),
                       __int_as_float(__builtin_amdgcn_ds_bpermute(a, __float_as_int(v.y))),
                       __int_as_float(__builtin_amdgcn_ds_bpermute(a, __float_as_int(v.z))),
                       __int_as_float(__builtin_amdgcn_ds_bpermute(a, __float_as_int(v.w))));
}
__device__ __forceinline__ bool wave_node_fetch(const HgKernelParams& kp, bool want, uint32_t node, NodePair& np) {
    const uint32_t lane = __lane_id();
    uint64_t m = wave_ballot(want);
    uint32_t slot = 0u, list = 0u, k = 0u;
    while (m != 0ull && k < 32u) {  // wave-uniform: one distinct record per iteration
        const uint32_t first = uint32_t(__builtin_amdgcn_readlane(int(node), int(__builtin_ctzll(m))));
        const bool same = want && node == first;
        m &= ~wave_ballot(same);
        slot = same ? k : slot;
        list = lane == k ? first : list;
        ++k;
    }
    if (m != 0ull) return false;
    const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (k <= 16u) {  // record j in lanes 4j .. 4j+3, 16 B each: one load instruction
        const uint32_t rec = bperm_u(lane >> 2, list);
        float4 a = z;
        if ((lane >> 2) < k) a = ld_off(kp.nodes, (rec << 6) + ((lane & 3u) << 4));
        const uint32_t s = slot << 2;
        np.q0 = bperm_f4(s, a);
        np.q1 = bperm_f4(s + 1u, a);
        np.q2 = bperm_f4(s + 2u, a);
        np.q3 = bperm_f4(s + 3u, a);
    } else {  // record j in lanes 2j, 2j+1: bytes 0-15 / 16-31 (first load), 32-47 / 48-63 (second)
        const uint32_t rec = bperm_u(lane >> 1, list);
        float4 a = z, b = z;
        if ((lane >> 1) < k) {
            const uint32_t off = (rec << 6) + ((lane & 1u) << 4);
            a = ld_off(kp.nodes, off);
            b = ld_off(kp.nodes, off + 32u);
        }
        const uint32_t s = slot << 1;
        np.q0 = bperm_f4(s, a);
        np.q1 = bperm_f4(s + 1u, a);
        np.q2 = bperm_f4(s, b);
        np.q3 = bperm_f4(s + 1u, b);
    }
    return true;
}
#endif

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
#if HG_PHASE_DETAIL == 2
    uint64_t tp = wave_clock();
#endif
    t.sph_t = HG_INF;
    t.sph = isect_spheres(kp, ray, t.sph_t);
#if HG_PHASE_DETAIL == 2
    if (kp.counters) tp = phase_mark(kp, 11, tp);
#endif
    t.best_t = t.sph_t;  // closestIntersection.rayT starts at the sphere hit (:381)
    t.best_u = 0.0f;
    t.best_v = 0.0f;
    t.best_tri = HG_NONE;
    t.best_mesh = 0;
    uint32_t culled = 0;
    const f3 winv = mk(rcp_exact(ray.d.x), rcp_exact(ray.d.y), rcp_exact(ray.d.z));
    t.live = mesh_live_mask(kp, ray.o, winv, t.best_t, culled);
#if HG_PHASE_DETAIL == 2
    if (kp.counters) tp = phase_mark(kp, 12, tp);
#endif
    c.aabb += 2 * culled;
    t.sp = 0;
    t.node = HG_NONE;
    const uint32_t nm = uint32_t(kp.n_meshes);
    t.mi = next_live_mesh(t.live, 0u, nm);
    f3 inv;
    if (t.mi < nm) mesh_local_ray<kMeshLds>(kp, ray, t.mi, t.lo, t.ld, inv, t.node);
#if HG_PHASE_DETAIL == 2
    if (kp.counters) {
        asm volatile("" : : "v"(t.node), "v"(t.lo.x), "v"(t.ld.x));  // keep the loads' wait inside this phase
        tp = phase_mark(kp, 13, tp);
    }
#endif
}

// One while-while round for the lanes with `act`: descend until each is at a leaf (or out of nodes), test that
// leaf, and move to the next live mesh when the current one is exhausted.
template <bool kMeshLds = false, class Stk>
__device__ __forceinline__ void trav_step(const HgKernelParams& kp, const Ray& ray, Trav& t, Counters& c,
                                          const Stk& stk, bool act, const LeafShare& ls) {
    // 1/ld (the same rcp_exact values mesh_local_ray computes) is not kept in Trav: live only during this round, it
    // stays out of the registers held across the streaming kernel's shading code
    const f3 inv = mk(rcp_exact(t.ld.x), rcp_exact(t.ld.y), rcp_exact(t.ld.z));
#if HG_PHASE_DETAIL == 3
    uint64_t tp = kp.counters ? wave_clock() : 0;
#endif
    const uint64_t act_mask = wave_ballot(act);  // act is fixed for the round
    const uint32_t dt = kp.descent_t;
    // lanes at an inner node (HG_NONE has the leaf bit): the wave descends while more than dt of them are left, or
    // while every active lane is still descending (relaxed while-while, as in isect_meshes)
    uint64_t dm = act_mask & wave_ballot(int32_t(t.node) >= 0);
    while (dm != 0ull && (uint32_t(__builtin_popcountll(dm)) > dt || dm == act_mask)) {
        c.node_rounds += wave_once();
#if HG_COHERENCE_STATS  // analysis builds: distinct node records among the loading lanes, into shade_detail[0..3]
        if (kp.counters) {  // buckets: 1-4 / 5-16 / 17-32 / more than 32 distinct records per node round
            uint64_t m = dm;
            uint32_t k = 0;
            while (m != 0ull) {
                const uint32_t first = uint32_t(__builtin_amdgcn_readlane(int(t.node), int(__builtin_ctzll(m))));
                m &= ~wave_ballot(t.node == first);
                ++k;
            }
            const int slot = k <= 4u ? 11 : k <= 16u ? 12 : k <= 32u ? 13 : 14;
            if (int(threadIdx.x & 63u) == __ffsll((unsigned long long)__ballot(1)) - 1)
                atomicAdd(kp.counters + slot, 1ull);
        }
#endif
#if (HG_QUAD_FETCH || HG_NODE_DEDUP) && !HG_NODE_CACHE
        const bool want = act && int32_t(t.node) >= 0;
        NodePair np;
#if HG_NODE_DEDUP
        const bool coop = wave_node_fetch(kp, want, t.node, np);
#else
        const bool coop = quad_node_fetch(kp, want, t.node, np.q0, np.q1, np.q2, np.q3);
#endif
        if (want) {
            if (!coop) np = node_pair(kp, t.node);
#else
        if (act && int32_t(t.node) >= 0) {
#endif
#if (HG_QUAD_FETCH || HG_NODE_DEDUP) && !HG_NODE_CACHE
#elif HG_NODE_CACHE
            // the BLAS tops (records [0, hot_records), hot_prefix) come from the wave's LDS copy
            const NodePair np = t.node < kp.hot_records
                                    ? node_pair_at(reinterpret_cast<const float4*>(hg_lds_stack + HG_STREAM_CACHE_ROW * 64u) +
                                                   4u * t.node)
                                    : node_pair(kp, t.node);
#else
            const NodePair np = node_pair(kp, t.node);
#endif
            const uint32_t refA = pair_ref_a(np), refB = pair_ref_b(np);
#if HG_NODE_PREFETCH
            // after all four loads have landed (vmcnt retires in order: a wait for a later load would include it)
            asm volatile("" : : "v"(np.q0.w), "v"(np.q1.w), "v"(np.q2.z), "v"(np.q3.y));
            node_prefetch(kp, refA, refB);
#endif
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
#if HG_PHASE_DETAIL == 3
    if (kp.counters) tp = phase_mark(kp, 11, tp);
#endif
    bool seq_leaf = true;  // the leaf's triangles tested by the lane itself, in order
#if HG_LEAF_DIST
    {
        const bool at_leaf = act && t.node != HG_NONE && (t.node & HG_LEAF_BIT);
        uint32_t first = 0u, n = 0u;
        if (at_leaf) {
            const uint2 lr = leaf_range(kp, t.node);
            first = lr.x;
            n = lr.y;
        }
        // distribute only when the longest leaf would take enough sequential rounds to pay for the exchange
        if (HG_LEAF_DIST_MIN <= 1 || uint32_t(__builtin_amdgcn_readlane(int(wave_incl_max(n)), 63)) >= HG_LEAF_DIST_MIN) {
            if (leaf_dist(kp, LeafRay{t.lo, t.ld, t.best_t, t.best_u, t.best_v, t.best_tri, t.best_mesh, t.mi}, c,
                          ls, first, n)) {
                if (at_leaf) t.node = t.sp > 0 ? stk.pop(t.sp) : HG_NONE;
                seq_leaf = false;
            }
        }
    }
#else
    (void)ls;
#endif
    if (seq_leaf && act && t.node != HG_NONE && (t.node & HG_LEAF_BIT)) {  // :404-420
        const uint2 leaf = leaf_range(kp, t.node);
        const uint32_t end = leaf.x + leaf.y;
#if HG_STREAM_TRI_PREFETCH
        float4 na, nb;
        float nc;
        tri_load(kp, leaf.x, na, nb, nc);
#endif
        for (uint32_t ti = leaf.x; ti < end; ++ti) {
            c.tri_rounds += wave_once();
#if HG_STREAM_TRI_PREFETCH  // the next triangle's loads go out before this one is tested
            const float4 a = na, b = nb;
            const float cz = nc;
            const uint32_t tn = ti + 1 < end ? ti + 1 : ti;
            tri_load(kp, tn, na, nb, nc);
#else
            float4 a, b;
            float cz;
            tri_load(kp, ti, a, b, cz);
#endif
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
#if HG_PHASE_DETAIL == 3
    if (kp.counters) tp = phase_mark(kp, 12, tp);
#endif
    if (act && t.node == HG_NONE) {
        const uint32_t nm = uint32_t(kp.n_meshes);
        t.mi = next_live_mesh(t.live, t.mi + 1u, nm);
        f3 inv_next;
        if (t.mi < nm) mesh_local_ray<kMeshLds>(kp, ray, t.mi, t.lo, t.ld, inv_next, t.node);
    }
#if HG_PHASE_DETAIL == 3
    if (kp.counters) {
        asm volatile("" : : "v"(t.node), "v"(t.lo.x), "v"(t.ld.x));
        tp = phase_mark(kp, 13, tp);
    }
#endif
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
#if HG_PINHOLE_FAST
    // Pinhole (disc radius 0): ap is (+-0, +-0, 0), the zeros' signs those of cos / sin.  Nothing below can see them
    // when the camera translation has no zero component (m[3] + (+-0) = m[3] in xform) and pf has no -0 component:
    // ndcx, ndcy are never -0 (x - 1 rounds an exact 0 to +0), so with vw, vh > 0 screen.x, .y are never -0 either
    // (+0 + -0 = +0; no sum underflows), and normalize / the focal distance > 0 keep the sign.  Then pf - (+-0) = pf,
    // and the focal sample and its sincos are skipped: the same bits.
    if (!(kp.focal_disc_radius == 0.0f && kp.cam[3] != 0.0f && kp.cam[7] != 0.0f && kp.cam[11] != 0.0f &&
          kp.vw > 0.0f && kp.vh > 0.0f && kp.near_ > 0.0f && kp.focal_dist > 0.0f))
#endif
    {
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

