/*
 * hg_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + cpu_baseline of bench.py).
 *
 * A deliberately literal, scalar, AoS restatement of the reference hot path:
 *   Assets/Scripts/Halogen Shaders/HalgoenCompute.compute   (kernel, lines cited per function)
 *   Assets/Scripts/Halogen Shaders/HalogenRandom.hlsl       (sampler)
 *   Assets/Scripts/Halogen Shaders/HalogenDefines.hlsl      (switches: importance sampling on, range 8,
 *                                                            PRNG override off, RR on)
 *   Assets/Scripts/Halogen Shaders/AccumulationShader.shader:27-34 (progressive blend)
 *   Assets/Scripts/BVHGenerator.cs                          (BLAS build, Unity Bounds semantics)
 * It follows the reference's control flow, including its quirks, and uses the
 * shared arithmetic spec include/hg_fmath.h for every non-basic operation.
 *
 * PARITY UNPINNED against reference outputs (none exist and the HLSL cannot run here); see hg_oracle.h.
 */
#include "hg_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "hg_fmath.h"

#ifndef HGO_STATS
#define HGO_STATS 0 /* 1: the stats build (diagnostic counts, see hgo_stack_stats) */
#endif

/* ------------------------------------------------------------------------------------------------
 * small vector helpers, literal HLSL semantics (no FMA contraction; compiled -ffp-contract=off)
 * ---------------------------------------------------------------------------------------------- */
typedef struct { float x, y, z; } f3;
static inline f3 v3(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline f3 add3(f3 a, f3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 sub3(f3 a, f3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 mul3(f3 a, f3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline f3 muls(f3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline f3 neg3(f3 a) { return v3(-a.x, -a.y, -a.z); }
static inline float dot3(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline f3 cross3(f3 a, f3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float length3(f3 a) { return __builtin_sqrtf(dot3(a, a)); }
static inline f3 normalize3(f3 a) { return muls(a, hg_rnorm(dot3(a, a))); }
static inline f3 lerp3(f3 a, f3 b, float s) { return add3(a, muls(sub3(b, a), s)); }
static inline f3 fromv(hg_vec3 a) { return v3(a.x, a.y, a.z); }
/* mul(M, float4(v, w)) with M a Unity column-major matrix: row r = M(r,0)v.x + M(r,1)v.y + M(r,2)v.z + M(r,3)w */
static inline f3 mat_mul(const hg_mat4* M, f3 v, float w) {
    const float* m = M->m;
    return v3(((m[0] * v.x + m[4] * v.y) + m[8] * v.z) + m[12] * w,
              ((m[1] * v.x + m[5] * v.y) + m[9] * v.z) + m[13] * w,
              ((m[2] * v.x + m[6] * v.y) + m[10] * v.z) + m[14] * w);
}
/* mul(float4(v, 0), M): row vector times matrix, column c = v.x M(0,c) + v.y M(1,c) + v.z M(2,c) + 0 M(3,c) */
static inline f3 vec_mul_mat(f3 v, const hg_mat4* M) {
    const float* m = M->m;
    return v3(((v.x * m[0] + v.y * m[1]) + v.z * m[2]) + 0.0f * m[3],
              ((v.x * m[4] + v.y * m[5]) + v.z * m[6]) + 0.0f * m[7],
              ((v.x * m[8] + v.y * m[9]) + v.z * m[10]) + 0.0f * m[11]);
}

/* ------------------------------------------------------------------------------------------------
 * Sampler — HalogenRandom.hlsl
 * ---------------------------------------------------------------------------------------------- */
/* Sobol direction numbers for dimensions 0..3 (HalogenRandom.hlsl:10-46).  Built here from the
 * Joe–Kuo construction (dim 0: van der Corput; dims 1..3 = Joe–Kuo d=2..4: (s,a,m) = (1,0,{1}),
 * (2,1,{1,3}), (3,1,{1,3,1})); tests/test_oracle_sampler.py checks the result against the reference's
 * literal table (tests/golden/sobol_table.json). */
static uint32_t g_sobol[4][32];
static pthread_once_t g_sobol_once = PTHREAD_ONCE_INIT;
static void build_sobol_table(void) {
    static const int s_[4] = {0, 1, 2, 3};
    static const uint32_t a_[4] = {0, 0, 1, 1};
    static const uint32_t m_[4][3] = {{0, 0, 0}, {1, 0, 0}, {1, 3, 0}, {1, 3, 1}};
    for (int k = 0; k < 32; k++) g_sobol[0][k] = 0x80000000u >> k;
    for (int d = 1; d < 4; d++) {
        int s = s_[d];
        for (int k = 0; k < 32; k++) {
            if (k < s) {
                g_sobol[d][k] = m_[d][k] << (31 - k);
            } else {
                uint32_t v = g_sobol[d][k - s] ^ (g_sobol[d][k - s] >> s);
                for (int i = 1; i < s; i++)
                    if ((a_[d] >> (s - 1 - i)) & 1u) v ^= g_sobol[d][k - i];
                g_sobol[d][k] = v;
            }
        }
    }
}
uint32_t hgo_sobol_table(uint32_t dim, uint32_t bit) {
    pthread_once(&g_sobol_once, build_sobol_table);
    return g_sobol[dim & 3][bit & 31];
}

/* u32_hash, HalogenRandom.hlsl:110-115 (PCG hash) */
uint32_t hgo_pcg_hash(uint32_t value) {
    uint32_t state = value * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
/* hash_combine, :131-133 */
uint32_t hgo_hash_combine(uint32_t seed, uint32_t v) { return seed ^ (v + (seed << 6) + (seed >> 2)); }

static inline uint32_t reversebits(uint32_t x) {
    x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
    x = ((x >> 8) & 0x00FF00FFu) | ((x & 0x00FF00FFu) << 8);
    return (x >> 16) | (x << 16);
}
/* owen_scramble, :140-161 */
uint32_t hgo_owen_scramble(uint32_t value, uint32_t seed) {
    uint32_t x = reversebits(value);
    x ^= x * 0x3d20adeau;
    x += seed;
    x *= (seed >> 16) | 1u;
    x ^= x * 0x05526c56u;
    x ^= x * 0x53a22864u;
    return reversebits(x);
}
/* sobol1d, :178-185 — literal 32-iteration loop */
uint32_t hgo_sobol1d(uint32_t index, uint32_t dim) {
    uint32_t X = 0;
    pthread_once(&g_sobol_once, build_sobol_table);
    for (int bit = 0; bit < 32; bit++) {
        uint32_t mask = (index >> bit) & 1u;
        X ^= mask * g_sobol[dim][bit];
    }
    return X;
}
/* u32_owen_scrambled_sobol, :203-209 */
uint32_t hgo_u32_owen_scrambled_sobol(uint32_t index, uint32_t dimension, uint32_t seed) {
    seed ^= hgo_pcg_hash(dimension);
    return hgo_owen_scramble(hgo_sobol1d(index, 0), hgo_pcg_hash(seed));
}
/* u32_2d_owen_scrambled_sobol, :215-228 */
void hgo_u32_2d_owen_scrambled_sobol(uint32_t index, uint32_t dimension, uint32_t seed, uint32_t out[2]) {
    seed ^= hgo_pcg_hash(dimension);
    uint32_t shuffled = hgo_owen_scramble(index, seed);
    uint32_t sx = hgo_sobol1d(shuffled, 0), sy = hgo_sobol1d(shuffled, 1);
    out[0] = hgo_owen_scramble(sx, hgo_hash_combine(seed, 0));
    out[1] = hgo_owen_scramble(sy, hgo_hash_combine(seed, 1));
}

/* Per-thread shader statics (HalogenRandom.hlsl:77-78, HalgoenCompute.compute:188-193) */
typedef struct {
    float ior;
    f3 absorption;
    int32_t priority;
    uint32_t materialID;
} medium_t;

typedef struct {
    const hgo_scene* sc;
    const hg_params* p;
    uint32_t frame;        /* FrameCount as uint */
    uint32_t dim_offset;   /* SobolDimensionOffset */
    uint32_t pixelID;      /* u32_hash(pixel index) */
    medium_t mstack[8];    /* participatingMediumStack */
    int msp;               /* mediumStackPointer */
    int tri_tests, aabb_tests; /* TriangleTests / AABBTests statics */
    hg_counters cnt;
#if HGO_STATS /* diagnostics of the stats build (merge_stats) */
    uint64_t st_overflow, st_visit[6];
    int32_t st_max;
#endif
} tstate;

#define ID_FOCAL 0u
#define ID_JITTER 1u
#define ID_ROUGH 2u
#define ID_PROPERTY 3u
#define ID_RR 4u
#define BOUNCE_INC 5u
#define INV_2_32 4294967296.0f

/* float_owen_scrambled_sobol, :252-259 (PRNG override off) */
static float float_sobol(tstate* t, uint32_t id) {
    return (float)hgo_u32_owen_scrambled_sobol(t->frame, t->dim_offset + id, t->pixelID) / INV_2_32;
}
/* float2_owen_scrambled_sobol, :261-268 */
static void float2_sobol(tstate* t, uint32_t id, float out[2]) {
    uint32_t u[2];
    hgo_u32_2d_owen_scrambled_sobol(t->frame, t->dim_offset + id, t->pixelID, u);
    out[0] = (float)u[0] / INV_2_32;
    out[1] = (float)u[1] / INV_2_32;
}

#define HLSL_PI (180.0f * HG_DEG2RAD) /* HalogenDefines.hlsl:12, PI = radians(180) */

/* get_random_unit_vector, :282-298 */
static f3 random_unit_vector(const float uv[2]) {
    float theta = uv[0] * 2.0f * HLSL_PI;
    float phi = hg_acosf(2.0f * uv[1] - 1.0f);
    float r = 1.0f;
    float sinTheta = hg_sinf(theta), cosTheta = hg_cosf(theta);
    float sinPhi = hg_sinf(phi), cosPhi = hg_cosf(phi);
    return v3(r * sinPhi * cosTheta, r * sinPhi * sinTheta, r * cosPhi);
}
/* get_random_point_circle, :303-308 */
static void random_point_circle(float radius, const float rd[2], float out[2]) {
    float theta = (rd[0] * 360.0f) * HG_DEG2RAD;
    float dist = rd[1];
    out[0] = hg_cosf(theta) * radius * dist;
    out[1] = hg_sinf(theta) * radius * dist;
}
/* arctanh :319-321, inverted_blackman_harris_cdf_approximation :328-330 */
float hgo_inverted_blackman_harris(float x) {
    float a = (x * 1.99221575606f) - 0.99610787803f;
    float at = 0.5f * hg_logf((1.0f + a) / (1.0f - a));
    return at / 6.24f;
}

/* ------------------------------------------------------------------------------------------------
 * Cubemap: TextureCube.SampleLevel (HC:201) with an integral level = bilinear within one mip, SEAMLESS as D3D10+
 * filters every cube map (and as the reference's asset is imported, seamlessCubemap: 1,
 * resting_place_4k.exr.meta:32): a footprint texel beyond a face edge is read from the adjacent face; at a cube
 * corner, where only three texels exist, the fourth is their average.  D3D face selection and (s, t) orientation,
 * faces +X,-X,+Y,-Y,+Z,-Z; texel centres at (i + 0.5) / size.  The kernel (hg_device.h sample_sky) is the same code.
 * ---------------------------------------------------------------------------------------------- */
/* Face frames: major axis M, s axis S, t axis T as integer unit vectors (sc = dot(d, S), tc = dot(d, T)). */
static const int CUBE_M[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
static const int CUBE_S[6][3] = {{0, 0, -1}, {0, 0, 1}, {1, 0, 0}, {1, 0, 0}, {1, 0, 0}, {-1, 0, 0}};
static const int CUBE_T[6][3] = {{0, -1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}, {0, -1, 0}, {0, -1, 0}};

/* Texel (i, j) of face f with i or j one step outside [0, size): the texel of the adjacent face that the extended
 * face plane crosses into.  Exact integer form: texel centres at odd coordinates of a cube spanning [-size, size]:
 * P = size M + (2i + 1 - size) S + (2j + 1 - size) T; the component of magnitude size + 1 names the new face; on it
 * a coordinate of magnitude size (the old face's plane) is the edge texel, any other c is texel (c + size - 1) / 2
 * (dividing the direction by (size + 1) / size moves a centre by less than half a texel). */
static void cube_adjacent(int f, int i, int j, int size, int* nf, int* ni, int* nj) {
    const int a = 2 * i + 1 - size, b = 2 * j + 1 - size;
    int P[3];
    for (int k = 0; k < 3; k++) P[k] = size * CUBE_M[f][k] + a * CUBE_S[f][k] + b * CUBE_T[f][k];
    int g = 0;
    for (int k = 0; k < 3; k++)
        if (P[k] == size + 1 || P[k] == -(size + 1)) g = 2 * k + (P[k] < 0 ? 1 : 0);
    int c[2];
    for (int e = 0; e < 2; e++) {
        const int* ax = e == 0 ? CUBE_S[g] : CUBE_T[g];
        const int v = P[0] * ax[0] + P[1] * ax[1] + P[2] * ax[2];
        c[e] = (v == size || v == -size) ? (v > 0 ? size - 1 : 0) : (v + size - 1) / 2;
    }
    *nf = g;
    *ni = c[0];
    *nj = c[1];
}

void hgo_cube_sample(const hgo_scene* sc, const float dir[3], int32_t level, float rgb[3]) {
    float x = dir[0], y = dir[1], z = dir[2];
    float ax = x < 0 ? -x : x, ay = y < 0 ? -y : y, az = z < 0 ? -z : z;
    int face;
    float sc_, tc, ma;
    if (az >= ax && az >= ay) {
        ma = az;
        if (z >= 0) { face = 4; sc_ = x; tc = -y; } else { face = 5; sc_ = -x; tc = -y; }
    } else if (ay >= ax) {
        ma = ay;
        if (y >= 0) { face = 2; sc_ = x; tc = z; } else { face = 3; sc_ = x; tc = -z; }
    } else {
        ma = ax;
        if (x >= 0) { face = 0; sc_ = -z; tc = -y; } else { face = 1; sc_ = z; tc = -y; }
    }
    if (level < 0) level = 0;
    if (level > sc->cube_mips - 1) level = sc->cube_mips - 1;
    int64_t off = 0;
    for (int m = 0; m < level; m++) {
        int64_t s = sc->cube_face_size >> m;
        if (s < 1) s = 1;
        off += 6 * s * s * 4;
    }
    int size = sc->cube_face_size >> level;
    if (size < 1) size = 1;
    const float* mip = sc->cube_texels + off;
    float s = (sc_ / ma + 1.0f) * 0.5f;
    float t = (tc / ma + 1.0f) * 0.5f;
    float u = s * (float)size - 0.5f, v = t * (float)size - 0.5f;
    float fu0 = __builtin_floorf(u), fv0 = __builtin_floorf(v);
    float fx = u - fu0, fy = v - fv0;
    const int xs[2] = {(int)fu0, (int)fu0 + 1}, ys[2] = {(int)fv0, (int)fv0 + 1};
    float tex[2][2][3]; /* [row][col][rgb] */
    int corner = -1;    /* footprint texel with both coordinates off the face */
    for (int r = 0; r < 2; r++) {
        for (int q = 0; q < 2; q++) {
            const int i = xs[q], j = ys[r];
            const int in_i = i >= 0 && i < size, in_j = j >= 0 && j < size;
            if (!in_i && !in_j) {
                corner = r * 2 + q;
                continue;
            }
            int f = face, ii = i, jj = j;
            if (!in_i || !in_j) cube_adjacent(face, i, j, size, &f, &ii, &jj);
            const float* p = mip + (((int64_t)f * size + jj) * size + ii) * 4;
            for (int c = 0; c < 3; c++) tex[r][q][c] = p[c];
        }
    }
    if (corner >= 0) { /* the average of the other three: same row, same column, diagonal */
        const int r = corner >> 1, q = corner & 1;
        for (int c = 0; c < 3; c++)
            tex[r][q][c] = ((tex[r][1 - q][c] + tex[1 - r][q][c]) + tex[1 - r][1 - q][c]) / 3.0f;
    }
    for (int c = 0; c < 3; c++) {
        float top = tex[0][0][c] * (1.0f - fx) + tex[0][1][c] * fx;
        float bot = tex[1][0][c] * (1.0f - fx) + tex[1][1][c] * fx;
        rgb[c] = top * (1.0f - fy) + bot * fy;
    }
}

/* Exposed for the adjacency unit test (tests/test_cubemap.py). */
void hgo_cube_adjacent(int32_t f, int32_t i, int32_t j, int32_t size, int32_t out[3]) {
    int nf, ni, nj;
    cube_adjacent(f, i, j, size, &nf, &ni, &nj);
    out[0] = nf;
    out[1] = ni;
    out[2] = nj;
}

/* sample_sky, :196-204.  level is already the int the reference passes. */
static f3 sample_sky(tstate* t, f3 dir, int level) {
    if (t->p->useEnvironmentCubemap > 0 && t->sc->cube_texels) {
        float d[3] = {dir.x, dir.y, dir.z}, rgb[3];
        hgo_cube_sample(t->sc, d, level, rgb);
        return v3(rgb[0], rgb[1], rgb[2]);
    }
    return v3(0, 0, 0);
}
/* int(round(DefaultHDRIMipLevel + accRough*8)) with the float->int conversion clamped */
static int sky_level(const hg_params* p, float accRough) {
    float lf = hg_roundf((float)p->defaultHDRIMipLevel + accRough * 8.0f);
    if (!(lf >= 0.0f)) return 0;
    if (lf > 64.0f) return 64;
    return (int)lf;
}

/* ------------------------------------------------------------------------------------------------
 * Intersection — HalgoenCompute.compute:244-485
 * ---------------------------------------------------------------------------------------------- */
typedef struct { f3 o, d; } ray_t;

typedef struct {
    float rayT;
    float orientation;
    f3 pos, normal;
    uint32_t material; /* index into MaterialList */
} hit_t;

/* ray_AABB_test, :244-259 (dir pre-inverted) */
static float ray_aabb(f3 A, f3 B, const ray_t* r) {
    f3 t1 = mul3(sub3(A, r->o), r->d);
    f3 t2 = mul3(sub3(B, r->o), r->d);
    float tMin = fminf(t1.x, t2.x);
    float tMax = fmaxf(t1.x, t2.x);
    tMin = fmaxf(tMin, fminf(t1.y, t2.y));
    tMax = fminf(tMax, fmaxf(t1.y, t2.y));
    tMin = fmaxf(tMin, fminf(t1.z, t2.z));
    tMax = fminf(tMax, fmaxf(t1.z, t2.z));
    return tMax > fmaxf(0.0f, tMin) ? tMin : HG_INF;
}

/* sphere_intersection, :266-303 */
static hit_t sphere_intersection(const ray_t* ray, const HalogenSphere* s) {
    hit_t h;
    memset(&h, 0, sizeof h);
    f3 shifted = sub3(ray->o, fromv(s->center));
    float b = 2.0f * dot3(shifted, ray->d);
    float c = dot3(shifted, shifted) - s->radius * s->radius;
    float disc = b * b - 4.0f * c;
    h.rayT = HG_INF;
    if (disc >= 0.0f) {
        float hd = (-b - __builtin_sqrtf(disc)) / 2.0f;
        h.orientation = 1.0f;
        if (hd < 0.0f) {
            hd = (-b + __builtin_sqrtf(disc)) / 2.0f;
            h.orientation = -1.0f;
        }
        h.rayT = hd;
        h.pos = add3(ray->o, muls(ray->d, hd));
        h.normal = muls(normalize3(sub3(h.pos, fromv(s->center))), h.orientation);
        h.material = s->materialIndex;
    }
    return h;
}

typedef struct {
    float rayT;
    float u, v;
    uint32_t mesh, tri;
    float orientation;
} tri_isect;

/* triangle_intersection_doublesided, :307-355 */
static tri_isect triangle_intersection(const ray_t* ray, const HalogenTriangle* tri) {
    tri_isect r;
    memset(&r, 0, sizeof r);
    r.rayT = HG_INF;
    f3 v0 = fromv(tri->pointA), v1 = fromv(tri->pointB), v2 = fromv(tri->pointC);
    f3 v0v1 = sub3(v1, v0), v0v2 = sub3(v2, v0);
    f3 pvec = cross3(ray->d, v0v2);
    float det = dot3(pvec, v0v1);
    if (fabsf(det) < 0.00000001f) return r;
    float inv = 1.0f / det;
    f3 tvec = sub3(ray->o, v0);
    float U = dot3(tvec, pvec) * inv;
    if (U < 0.0f || U > 1.0f) return r;
    f3 qvec = cross3(tvec, v0v1);
    float V = dot3(ray->d, qvec) * inv;
    if (V < 0.0f || U + V > 1.0f) return r;
    float t = dot3(v0v2, qvec) * inv;
    if (t > 0.0f) {
        r.u = U;
        r.v = V;
        r.rayT = t;
        r.orientation = det > 0.0f ? 1.0f : (det < 0.0f ? -1.0f : 0.0f);
    }
    return r;
}

/* get_ray_scene_intersection_sphere, :357-376 */
static void scene_isect_spheres(tstate* t, const ray_t* ray, hit_t* closest) {
    float closestDistance = closest->rayT;
    ray_t pre = *ray;
    pre.d = v3(1.0f / ray->d.x, 1.0f / ray->d.y, 1.0f / ray->d.z);
    int n = (int)t->p->bufferCounts.x;
    for (int i = 0; i < n; i++) {
        const HalogenSphere* s = &t->sc->spheres[i];
        t->cnt.sphere_tests++;
        if (ray_aabb(fromv(s->boundingCornerA), fromv(s->boundingCornerB), &pre) < t->p->viewParameters.w) {
            hit_t h = sphere_intersection(ray, s);
            if (h.rayT < closestDistance && h.rayT > 0.0001f) {
                *closest = h;
                closestDistance = h.rayT;
            }
        }
    }
}

#define NODE_STACK 64 /* reference: int NodeStack[32] (:397); 33 can be needed at depth cap 32, see DESIGN.md */
#define REF_NODE_STACK 32 /* the reference's array size: a push at index >= 32 is out of bounds in HC:397-444 */

/* Diagnostics (test infra; tools/stack_depth.py, tools/visit_stats.py, tests/test_oracle.py): compiled only into the
 * stats build (HGO_STATS=1, build/libhgoracle_stats.so).  The plain build, which the parity tests and bench.py's
 * cpu_baseline load, has none of it in the traversal.  The stats build counts per thread (tstate) and merges once per
 * render job, so even there no shared cache line sits in the traversal loop.
 *   stack: mesh traversals whose stack would outgrow the reference's NodeStack[32], and the deepest stack seen;
 *   visits: inner-node visits by how many of the two children the exact test keeps (t < closest), for mesh roots and
 *           for deeper nodes: [root 0/1/2, inner 0/1/2].
 * All since the last reset (hgo_stack_stats / hgo_visit_stats with reset=1). */
static pthread_mutex_t g_stats_mu = PTHREAD_MUTEX_INITIALIZER;
static uint64_t g_stack_overflow_traversals;
static int32_t g_stack_max;
static uint64_t g_visit_ok[6];
int hgo_stats_build(void) { return HGO_STATS; }
void hgo_stack_stats(uint64_t* overflow_traversals, int32_t* max_depth, int32_t reset) {
    pthread_mutex_lock(&g_stats_mu);
    if (overflow_traversals) *overflow_traversals = g_stack_overflow_traversals;
    if (max_depth) *max_depth = HGO_STATS ? g_stack_max : -1;
    if (reset) {
        g_stack_overflow_traversals = 0;
        g_stack_max = 0;
    }
    pthread_mutex_unlock(&g_stats_mu);
}
void hgo_visit_stats(uint64_t out[6], int32_t reset) {
    pthread_mutex_lock(&g_stats_mu);
    for (int k = 0; k < 6; ++k) {
        if (out) out[k] = g_visit_ok[k];
        if (reset) g_visit_ok[k] = 0;
    }
    pthread_mutex_unlock(&g_stats_mu);
}
#if HGO_STATS
/* the popped node was the mesh's root: the stack was empty after its pop and nothing had been pushed before */
static int stack_is_root(int sp, int high) { return sp == 0 && high == 1; }
#endif
/* a thread's counts into the globals (once per render job / traced pixel) */
static void merge_stats(const tstate* t) {
#if HGO_STATS
    pthread_mutex_lock(&g_stats_mu);
    g_stack_overflow_traversals += t->st_overflow;
    if (t->st_max > g_stack_max) g_stack_max = t->st_max;
    for (int k = 0; k < 6; ++k) g_visit_ok[k] += t->st_visit[k];
    pthread_mutex_unlock(&g_stats_mu);
#else
    (void)t;
#endif
}

/* get_ray_scene_intersection_mesh, :378-472 */
static void scene_isect_meshes(tstate* t, const ray_t* ray, hit_t* closestHit) {
    const hgo_scene* sc = t->sc;
    tri_isect closest;
    memset(&closest, 0, sizeof closest);
    closest.rayT = closestHit->rayT;
    const float eps = 0.0001f;
    int n = (int)t->p->bufferCounts.y;
    for (int i = 0; i < n; i++) {
        const HalogenMeshData* md = &sc->meshes[i];
        t->cnt.mesh_visits++;
        ray_t local;
        local.o = mat_mul(&md->worldToLocal, ray->o, 1.0f);
        local.d = mat_mul(&md->worldToLocal, ray->d, 0.0f);
        ray_t pre = local;
        pre.d = v3(1.0f / local.d.x, 1.0f / local.d.y, 1.0f / local.d.z);
        uint32_t stack[NODE_STACK];
        int sp = 0;
#if HGO_STATS
        int high = 1;
#endif
        stack[sp++] = md->accelerationBufferOffset;
        while (sp > 0) {
#if HGO_STATS
            if (sp > high) high = sp;
#endif
            const BVHEntry* node = &sc->blas[stack[--sp]];
            if (node->triangleCount > 0) {
                for (uint32_t k = 0; k < node->triangleCount; k++) {
                    tri_isect is = triangle_intersection(&local, &sc->triangles[k + md->triangleBufferOffset + node->indexA]);
                    t->tri_tests++;
                    t->cnt.tri_tests++;
                    if (is.rayT > eps && is.rayT < closest.rayT) {
                        closest = is;
                        closest.mesh = (uint32_t)i;
                        closest.tri = k + node->indexA;
                    }
                }
            } else {
                uint32_t ia = md->accelerationBufferOffset + node->indexA;
                const BVHEntry* A = &sc->blas[ia];
                const BVHEntry* B = &sc->blas[ia + 1];
                float dA = ray_aabb(fromv(A->boundingCornerA), fromv(A->boundingCornerB), &pre);
                float dB = ray_aabb(fromv(B->boundingCornerA), fromv(B->boundingCornerB), &pre);
                t->aabb_tests += 2;
                t->cnt.aabb_tests += 2;
#if HGO_STATS
                t->st_visit[(stack_is_root(sp, high) ? 0 : 3) + (dA < closest.rayT) + (dB < closest.rayT)]++;
#endif
                /* pushes beyond NODE_STACK are dropped; hg_upload_scene rejects trees deep enough to
                 * reach that, so this is a guard, not behaviour */
                if (dB < dA) {
                    if (dA < closest.rayT && sp < NODE_STACK) stack[sp++] = ia;
                    if (dB < closest.rayT && sp < NODE_STACK) stack[sp++] = ia + 1;
                } else {
                    if (dB < closest.rayT && sp < NODE_STACK) stack[sp++] = ia + 1;
                    if (dA < closest.rayT && sp < NODE_STACK) stack[sp++] = ia;
                }
            }
        }
#if HGO_STATS
        if (high > REF_NODE_STACK) t->st_overflow++;
        if (high > t->st_max) t->st_max = high;
#endif
    }
    if (closest.rayT < (closestHit->rayT - eps) && closest.rayT < t->p->viewParameters.w) {
        const HalogenMeshData* md = &sc->meshes[closest.mesh];
        const HalogenTriangle* tri = &sc->triangles[md->triangleBufferOffset + closest.tri];
        closestHit->rayT = closest.rayT;
        closestHit->material = md->materialIndex;
        closestHit->orientation = closest.orientation;
        f3 n0 = fromv(tri->normalA), n1 = fromv(tri->normalB), n2 = fromv(tri->normalC);
        f3 nrm = add3(add3(n0, muls(sub3(n1, n0), closest.u)), muls(sub3(n2, n0), closest.v));
        nrm = muls(nrm, closest.orientation);
        nrm = normalize3(vec_mul_mat(nrm, &md->worldToLocal));
        closestHit->normal = nrm;
        closestHit->pos = add3(ray->o, muls(ray->d, closest.rayT));
    }
}

/* get_ray_intersection, :474-485 */
static hit_t get_ray_intersection(tstate* t, const ray_t* ray) {
    hit_t h;
    memset(&h, 0, sizeof h);
    h.rayT = HG_INF;
    t->cnt.rays++;
    scene_isect_spheres(t, ray, &h);
    scene_isect_meshes(t, ray, &h);
    return h;
}

/* ------------------------------------------------------------------------------------------------
 * BSDF and medium stack — :491-817
 * ---------------------------------------------------------------------------------------------- */
static f3 lambert_scatter(f3 n, f3 rv) { /* :491-501 */
    f3 p = add3(rv, n);
    if (length3(p) < 1e-8f) p = n;
    return normalize3(p);
}
static f3 specular_scatter(f3 i, f3 n) { return sub3(i, muls(n, 2.0f * dot3(i, n))); } /* :506-509 */

static float schlick_adjusted(float n1, float n2, f3 normal, f3 incident, float minS, float maxS) { /* :519-540 */
    float r0 = (n1 - n2) / (n1 + n2);
    r0 *= r0;
    float cosX = -dot3(normal, incident);
    if (n1 > n2) {
        float n = n1 / n2;
        float sinT2 = n * n * (1.0f - cosX * cosX);
        if (sinT2 > 1.0f) return maxS;
        cosX = __builtin_sqrtf(1.0f - sinT2);
    }
    float x = 1.0f - cosX;
    float ret = r0 + (1.0f - r0) * x * x * x * x * x;
    return minS + ret * (maxS - minS);
}

static f3 refract_tir(f3 incident, f3 normal, float n1, float n2, int* tir) { /* :557-572 */
    float cos_theta = fminf(dot3(neg3(incident), normal), 1.0f);
    float sin_theta = __builtin_sqrtf(1.0f - cos_theta * cos_theta);
    float n12 = n1 / n2;
    if (n12 * sin_theta > 1.0f) {
        *tir = 1;
        return specular_scatter(incident, normal);
    }
    f3 perp = muls(add3(incident, muls(normal, cos_theta)), n12);
    float lp = length3(perp);
    f3 par = muls(normal, -__builtin_sqrtf(fabsf(1.0f - lp * lp)));
    return add3(perp, par);
}

static medium_t material_medium(const PackedHalogenMaterial* m) {
    medium_t r;
    r.ior = m->rayMedium.indexOfRefraction;
    r.absorption = fromv(m->rayMedium.absorption);
    r.priority = m->rayMedium.priority;
    r.materialID = m->rayMedium.materialID;
    return r;
}
static medium_t empty_medium(void) { /* :80-88 (priority 1.#INF -> int is never read) */
    medium_t r;
    r.ior = 1.0f;
    r.absorption = v3(0, 0, 0);
    r.priority = 0x7fffffff;
    r.materialID = 0xFFFFFFFFu;
    return r;
}

static void add_to_medium_stack(tstate* t, medium_t m) { /* :582-622 */
    if (t->msp == 0) {
        t->mstack[t->msp++] = m;
        return;
    }
    int ins = t->msp;
    if (m.priority > t->mstack[t->msp - 1].priority) {
        for (int i = t->msp - 1; i >= 0; i--) {
            if (m.priority < t->mstack[i].priority) { ins = i + 1; break; }
        }
        if (ins == t->msp) ins = 0;
    }
    if (t->msp >= 8) return; /* reference: unhandled overflow (UB); the build drops the push */
    if (ins != t->msp) {
        for (int i = t->msp - 1; i >= ins; i--) t->mstack[i + 1] = t->mstack[i];
        t->msp++;
        t->mstack[ins] = m;
    } else {
        t->mstack[t->msp++] = m;
    }
}
static void pop_from_medium_stack(tstate* t, uint32_t id) { /* :627-642 */
    for (int i = 0; i < t->msp; i++) {
        if (t->mstack[i].materialID == id) {
            for (int k = i + 1; k < t->msp; k++) t->mstack[k - 1] = t->mstack[k];
            t->msp--;
            return;
        }
    }
}
static medium_t top_medium(tstate* t) { return t->msp > 0 ? t->mstack[t->msp - 1] : empty_medium(); } /* :647-654 */
static int true_medium_hit(tstate* t, int32_t prio) { /* :656-665 */
    if (t->msp == 0) return 1;
    return prio <= t->mstack[t->msp - 1].priority;
}

/* material_BRDF, :672-741 */
static f3 material_brdf(tstate* t, ray_t* ray, const hit_t* hit, medium_t cur, medium_t hm, uint32_t* bounceType) {
    const PackedHalogenMaterial* mat = &t->sc->materials[hit->material];
    f3 att = v3(1, 1, 1);
    ray->o = hit->pos;
    float rr[2], pr[2];
    float2_sobol(t, ID_ROUGH, rr);
    float2_sobol(t, ID_PROPERTY, pr);
    f3 rrv = random_unit_vector(rr);
    int do_refraction = pr[0] > mat->albedo.w;
    float spec_rand = pr[1];
    float rough2 = mat->roughness * mat->roughness;
    if (!do_refraction) {
        att = v3(mat->albedo.x, mat->albedo.y, mat->albedo.z);
        f3 diffuseDir = lambert_scatter(hit->normal, rrv);
        float thr = (mat->metallic > 0.0f) ? schlick_adjusted(cur.ior, hm.ior, hit->normal, ray->d, mat->metallic, 1.0f)
                                           : mat->metallic;
        int spec = spec_rand < thr;
        *bounceType = spec ? 1u : 0u;
        if (spec) {
            f3 sd = specular_scatter(ray->d, hit->normal);
            sd = lerp3(sd, diffuseDir, rough2);
            att = v3(mat->specularAlbedo.x, mat->specularAlbedo.y, mat->specularAlbedo.z);
            ray->d = sd;
        } else {
            ray->d = diffuseDir;
        }
        ray->o = add3(hit->pos, muls(hit->normal, 0.0001f));
    } else {
        *bounceType = 2u;
        att = v3(1, 1, 1);
        int tir = 0;
        ray->d = refract_tir(ray->d, hit->normal, cur.ior, hm.ior, &tir);
        if (tir) {
            f3 dd = lambert_scatter(hit->normal, rrv);
            ray->d = lerp3(ray->d, dd, rough2);
            ray->o = sub3(hit->pos, muls(hit->normal, 0.0001f));
        } else {
            f3 dd = lambert_scatter(neg3(hit->normal), rrv);
            ray->d = lerp3(ray->d, dd, rough2);
            ray->o = sub3(hit->pos, muls(hit->normal, 0.0001f));
        }
    }
    ray->d = normalize3(ray->d);
    return att;
}

/* evaluate_material_hit, :743-817 */
static f3 evaluate_material_hit(tstate* t, ray_t* ray, const hit_t* hit, uint32_t bounceTypes[3]) {
    const PackedHalogenMaterial* mat = &t->sc->materials[hit->material];
    medium_t internal = material_medium(mat);
    f3 att = v3(1, 1, 1);
    medium_t cur, hm;
    int trueHit = 1;
    if (internal.priority >= 0) {
        trueHit = true_medium_hit(t, internal.priority);
        if (hit->orientation == 1.0f) {
            cur = top_medium(t);
            hm = internal;
            add_to_medium_stack(t, hm);
        } else {
            if (t->msp == 0) cur = internal;
            else cur = top_medium(t);
            pop_from_medium_stack(t, internal.materialID);
            hm = top_medium(t);
        }
    } else {
        if (hit->orientation == 1.0f) {
            cur = top_medium(t);
            hm = internal;
        } else {
            cur = internal;
            hm = top_medium(t);
        }
    }
    if (trueHit) {
        uint32_t bt = 0;
        att = material_brdf(t, ray, hit, cur, hm, &bt);
        bounceTypes[bt]++;
        if (hit->orientation > 0.0f && bt != 2u) pop_from_medium_stack(t, internal.materialID);
    } else {
        ray->o = sub3(hit->pos, muls(hit->normal, 0.0001f));
        att = v3(1, 1, 1);
        bounceTypes[2]++;
    }
    if (cur.materialID != 0xFFFFFFFFu) {
        att = v3(att.x * hg_expf(-cur.absorption.x * hit->rayT), att.y * hg_expf(-cur.absorption.y * hit->rayT),
                 att.z * hg_expf(-cur.absorption.z * hit->rayT));
    }
    return att;
}

/* trace_ray, :876-950 */
static f3 trace_ray(tstate* t, ray_t ray) {
    const hg_params* p = t->p;
    f3 acc = v3(0, 0, 0), thr = v3(1, 1, 1);
    float accRough = 0.0f;
    uint32_t bt[3] = {0, 0, 0};
    for (uint32_t it = 0; it <= p->maxBounces; it++) {
        if (bt[0] > p->maxDiffuseBounces || bt[1] > p->maxGlossyBounces || bt[2] > p->maxTransmissionBounces) break;
        hit_t hit = get_ray_intersection(t, &ray);
        if (hit.rayT < p->viewParameters.w) {
            const PackedHalogenMaterial* mat = &t->sc->materials[hit.material];
            t->cnt.hits++;
            f3 em = muls(v3(mat->emissive.x, mat->emissive.y, mat->emissive.z), mat->emissive.w);
            acc = add3(acc, mul3(em, thr));
            f3 att = evaluate_material_hit(t, &ray, &hit, bt);
            thr = mul3(thr, att);
            accRough += mat->roughness * thr.x; /* float3 -> float truncation (:911) */
            float rr = float_sobol(t, ID_RR);
            t->dim_offset += BOUNCE_INC;
            float contribution = fmaxf(fmaxf(thr.x, thr.y), thr.z);
            if (rr > contribution) break;
            thr = muls(thr, 1.0f / contribution);
        } else {
            if (it == 0) t->cnt.primary_misses++; /* the camera ray hit nothing (diagnostic, not in the reference) */
            acc = add3(acc, mul3(sample_sky(t, ray.d, sky_level(p, accRough)), thr));
            break;
        }
    }
    return acc;
}

/* trace_ray_debug, :952-982 (and the debug colour helpers :819-863) */
static f3 trace_ray_debug(tstate* t, ray_t ray) {
    const hg_params* p = t->p;
    t->tri_tests = 0;
    t->aabb_tests = 0;
    hit_t hit;
    switch (p->halogenDebugMode) {
        default:
            return v3(0, 0, 0);
        case 1:
            hit = get_ray_intersection(t, &ray);
            if (hit.rayT < p->viewParameters.w) {
                const PackedHalogenMaterial* m = &t->sc->materials[hit.material];
                return v3(m->albedo.x, m->albedo.y, m->albedo.z);
            }
            return sample_sky(t, ray.d, p->defaultHDRIMipLevel);
        case 2:
            hit = get_ray_intersection(t, &ray);
            if (hit.rayT < p->viewParameters.w)
                return v3((hit.normal.x + 1.0f) / 2.0f, (hit.normal.y + 1.0f) / 2.0f, (hit.normal.z + 1.0f) / 2.0f);
            return sample_sky(t, ray.d, p->defaultHDRIMipLevel);
        case 3:
            trace_ray(t, ray);
            if ((uint32_t)t->tri_tests > p->triangleDebugDisplayRange) return v3(1, 1, 1);
            return v3((float)t->tri_tests / (float)p->triangleDebugDisplayRange, 0, 0);
        case 4:
            trace_ray(t, ray);
            if ((uint32_t)t->aabb_tests > p->boxDebugDisplayRange) return v3(1, 1, 1);
            return v3((float)t->aabb_tests / (float)p->boxDebugDisplayRange, 0, 0);
        case 5:
            trace_ray(t, ray);
            if ((uint32_t)t->tri_tests > p->triangleDebugDisplayRange ||
                (uint32_t)t->aabb_tests > p->boxDebugDisplayRange)
                return v3(1, 1, 1);
            return v3((float)t->tri_tests / (float)p->triangleDebugDisplayRange, 0,
                      (float)t->aabb_tests / (float)p->boxDebugDisplayRange);
    }
}

/* get_ray_jitter :984-994, get_ray :996-1013 */
static ray_t get_ray(tstate* t, float ndcx, float ndcy) {
    const hg_params* p = t->p;
    const float W = p->screenParameters.x, H = p->screenParameters.y;
    const float vw = p->viewParameters.x, vh = p->viewParameters.y, near = p->viewParameters.z;
    float focalDiscRadius = hg_tanf(p->focalConeAngle * HG_DEG2RAD) * near;
    float fd[2], circ[2];
    float2_sobol(t, ID_FOCAL, fd);
    random_point_circle(focalDiscRadius, fd, circ);
    f3 ap = v3(circ[0], circ[1], 0.0f);
    f3 screen = v3(ndcx * vw, ndcy * vh, 1.0f * near);
    /* jitter */
    float psx = (vw * 2.0f) / W, psy = (vh * 2.0f) / H;
    float jr[2];
    float2_sobol(t, ID_JITTER, jr);
    float jx = (hgo_inverted_blackman_harris(jr[0]) - 0.5f) * 2.0f * p->filterRadius * psx;
    float jy = (hgo_inverted_blackman_harris(jr[1]) - 0.5f) * 2.0f * p->filterRadius * psy;
    screen = add3(screen, v3(jx, jy, 0.0f));
    f3 pf = muls(normalize3(screen), p->focalPlaneDistance);
    f3 csd = normalize3(sub3(pf, ap));
    ray_t r;
    r.o = mat_mul(&p->camLocalToWorld, ap, 1.0f);
    r.d = normalize3(mat_mul(&p->camLocalToWorld, csd, 0.0f));
    return r;
}

/* HalogenCompute body, :1015-1062, for one pixel and one FrameCount.  Returns RayColor/SPP. */
static f3 halogen_compute_pixel(tstate* t, uint32_t x, uint32_t y) {
    const hg_params* p = t->p;
    const float W = p->screenParameters.x, H = p->screenParameters.y;
    float uvx = (float)x / W, uvy = (float)y / H;
    float ndcx = uvx * 2.0f - 1.0f, ndcy = uvy * 2.0f - 1.0f;
    t->pixelID = hgo_pcg_hash(x + y * (uint32_t)W);
    t->dim_offset = 0;
    t->msp = 0;
    t->tri_tests = t->aabb_tests = 0;
    f3 color = v3(0, 0, 0);
    for (uint32_t s = 0; s < p->samplesPerPixel; s++) {
        ray_t r = get_ray(t, ndcx, ndcy);
        t->cnt.paths++;
        if (p->halogenDebugMode < 1) color = add3(color, trace_ray(t, r));
        else color = add3(color, trace_ray_debug(t, r));
    }
    float spp = (float)p->samplesPerPixel;
    return v3(color.x / spp, color.y / spp, color.z / spp);
}

void hgo_trace_pixel(const hgo_scene* scene, const hg_params* params, uint32_t x, uint32_t y, int32_t frame,
                     float rgb[3], hg_counters* counters) {
    tstate t;
    memset(&t, 0, sizeof t);
    t.sc = scene;
    t.p = params;
    t.frame = (uint32_t)frame;
    f3 c = halogen_compute_pixel(&t, x, y);
    merge_stats(&t);
    rgb[0] = c.x;
    rgb[1] = c.y;
    rgb[2] = c.z;
    if (counters) {
        counters->paths += t.cnt.paths;
        counters->rays += t.cnt.rays;
        counters->tri_tests += t.cnt.tri_tests;
        counters->aabb_tests += t.cnt.aabb_tests;
        counters->mesh_visits += t.cnt.mesh_visits;
        counters->sphere_tests += t.cnt.sphere_tests;
        counters->hits += t.cnt.hits;
        counters->primary_misses += t.cnt.primary_misses;
    }
}

/* ------------------------------------------------------------------------------------------------
 * Frame loop + progressive accumulation (RP:324-347, AccumulationShader.shader:27-34)
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
    const hgo_scene* sc;
    const hg_params* p;
    int32_t n_frames, accumulate;
    float* acc;
    int64_t begin, end;
    int32_t tid, nthreads;
    hg_counters cnt;
} job_t;

static void* render_job(void* arg) {
    job_t* j = (job_t*)arg;
    const hg_params* p = j->p;
    const uint32_t W = (uint32_t)p->screenParameters.x;
    tstate t;
    memset(&t, 0, sizeof t);
    t.sc = j->sc;
    t.p = p;
    /* rows interleaved across threads */
    for (int64_t pix = j->begin; pix < j->end; pix++) {
        uint32_t y = (uint32_t)(pix / W), x = (uint32_t)(pix % W);
        if ((int64_t)(y % (uint32_t)j->nthreads) != j->tid) continue;
        float* a = j->acc + pix * 4;
        for (int32_t f = 0; f < j->n_frames; f++) {
            int32_t fc = j->accumulate ? p->frameCount + f : 1;
            t.frame = (uint32_t)fc;
            f3 c = halogen_compute_pixel(&t, x, y);
            float nw[4] = {c.x, c.y, c.z, 1.0f};
            if (j->accumulate) {
                float w = 1.0f / (float)fc;
                for (int k = 0; k < 4; k++) a[k] = a[k] * (1.0f - w) + nw[k] * w;
            } else {
                for (int k = 0; k < 4; k++) a[k] = nw[k];
            }
        }
    }
    j->cnt = t.cnt;
    merge_stats(&t);
    return NULL;
}

int hgo_render(const hgo_scene* scene, const hg_params* params, int32_t n_frames, int32_t accumulate, float* acc,
               int64_t pix_begin, int64_t pix_end, int32_t n_threads, hg_counters* counters) {
    if (!scene || !params || !acc || n_threads < 1 || n_threads > 1024) return -1;
    pthread_once(&g_sobol_once, build_sobol_table);
    job_t* jobs = (job_t*)calloc((size_t)n_threads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return -3; }
    for (int i = 0; i < n_threads; i++) {
        jobs[i].sc = scene;
        jobs[i].p = params;
        jobs[i].n_frames = n_frames;
        jobs[i].accumulate = accumulate;
        jobs[i].acc = acc;
        jobs[i].begin = pix_begin;
        jobs[i].end = pix_end;
        jobs[i].tid = i;
        jobs[i].nthreads = n_threads;
        if (n_threads > 1) pthread_create(&th[i], NULL, render_job, &jobs[i]);
    }
    if (n_threads == 1) render_job(&jobs[0]);
    else for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
    if (counters) {
        for (int i = 0; i < n_threads; i++) {
            counters->paths += jobs[i].cnt.paths;
            counters->rays += jobs[i].cnt.rays;
            counters->tri_tests += jobs[i].cnt.tri_tests;
            counters->aabb_tests += jobs[i].cnt.aabb_tests;
            counters->mesh_visits += jobs[i].cnt.mesh_visits;
            counters->sphere_tests += jobs[i].cnt.sphere_tests;
            counters->hits += jobs[i].cnt.hits;
            counters->primary_misses += jobs[i].cnt.primary_misses;
        }
    }
    free(jobs);
    free(th);
    return 0;
}

/* ------------------------------------------------------------------------------------------------
 * Per-stage KATs
 * ---------------------------------------------------------------------------------------------- */
float hgo_sphere_t(const float o[3], const float d[3], const float c[3], float r) {
    HalogenSphere s;
    memset(&s, 0, sizeof s);
    s.center.x = c[0]; s.center.y = c[1]; s.center.z = c[2];
    s.radius = r;
    ray_t ray = {v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2])};
    return sphere_intersection(&ray, &s).rayT;
}
float hgo_triangle_t(const float o[3], const float d[3], const float a[3], const float b[3], const float c[3],
                     float* u, float* v, float* orientation) {
    HalogenTriangle tri;
    memset(&tri, 0, sizeof tri);
    tri.pointA.x = a[0]; tri.pointA.y = a[1]; tri.pointA.z = a[2];
    tri.pointB.x = b[0]; tri.pointB.y = b[1]; tri.pointB.z = b[2];
    tri.pointC.x = c[0]; tri.pointC.y = c[1]; tri.pointC.z = c[2];
    ray_t ray = {v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2])};
    tri_isect is = triangle_intersection(&ray, &tri);
    if (u) *u = is.u;
    if (v) *v = is.v;
    if (orientation) *orientation = is.orientation;
    return is.rayT;
}
float hgo_aabb_t(const float a[3], const float b[3], const float o[3], const float inv_d[3]) {
    ray_t r = {v3(o[0], o[1], o[2]), v3(inv_d[0], inv_d[1], inv_d[2])};
    return ray_aabb(v3(a[0], a[1], a[2]), v3(b[0], b[1], b[2]), &r);
}

/* ------------------------------------------------------------------------------------------------
 * BVHGenerator.GenerateMeshBVH (BVHGenerator.cs:13-134) with UnityEngine.Bounds arithmetic
 * (centre/extents storage: SetMinMax -> extents=(max-min)*0.5, center=min+extents; min=center-extents,
 * max=center+extents; size=extents*2; the thin-box pad `bounds.max += one*1e-5` re-runs SetMinMax).
 * ---------------------------------------------------------------------------------------------- */
typedef struct { float c[3], e[3]; } ubounds;
static ubounds ub_setminmax(const float mn[3], const float mx[3]) {
    ubounds b;
    for (int k = 0; k < 3; k++) {
        b.e[k] = (mx[k] - mn[k]) * 0.5f;
        b.c[k] = mn[k] + b.e[k];
    }
    return b;
}
static void ub_min(const ubounds* b, float out[3]) { for (int k = 0; k < 3; k++) out[k] = b->c[k] - b->e[k]; }
static void ub_max(const ubounds* b, float out[3]) { for (int k = 0; k < 3; k++) out[k] = b->c[k] + b->e[k]; }

static const float AABB_EPS = 0.00001f; /* RayTracingMesh.AABBEpsilon (RayTracingMesh.cs:11) */

/* calculateBounds, BVHGenerator.cs:154-186 */
static ubounds calc_bounds(uint32_t start, uint32_t count, const int32_t* idx, const float* V) {
    float mn[3] = {HG_INF, HG_INF, HG_INF}, mx[3] = {-HG_INF, -HG_INF, -HG_INF};
    for (uint32_t i = start; i < start + count; i++) {
        for (int c = 0; c < 3; c++) {
            const float* p = V + 3 * (int64_t)idx[3 * (int64_t)i + c];
            for (int k = 0; k < 3; k++) mn[k] = (mn[k] < p[k]) ? mn[k] : p[k]; /* Mathf.Min: a < b ? a : b */
        }
        for (int c = 0; c < 3; c++) {
            const float* p = V + 3 * (int64_t)idx[3 * (int64_t)i + c];
            for (int k = 0; k < 3; k++) mx[k] = (mx[k] > p[k]) ? mx[k] : p[k]; /* Mathf.Max: a > b ? a : b */
        }
    }
    ubounds b = ub_setminmax(mn, mx);
    if (b.e[0] * 2.0f < AABB_EPS || b.e[1] * 2.0f < AABB_EPS || b.e[2] * 2.0f < AABB_EPS) {
        float nmx[3], nmn[3];
        ub_max(&b, nmx);
        for (int k = 0; k < 3; k++) nmx[k] = nmx[k] + AABB_EPS * 1.0f;
        ub_min(&b, nmn);
        b = ub_setminmax(nmn, nmx);
    }
    return b;
}

int64_t hgo_build_blas(const float* V, int32_t n_vertices, int32_t* idx, int32_t n_tris, const float root_min[3],
                       const float root_max[3], int32_t max_depth, BVHEntry* out, int64_t max_nodes) {
    (void)n_vertices;
    if (n_tris < 0 || !idx || !V) return -1;
    /* worst case node count: 2*n_tris - 1 + 1 */
    int64_t cap = 2 * (int64_t)n_tris + 2;
    BVHEntry* nodes = (BVHEntry*)malloc((size_t)cap * sizeof(BVHEntry));
    float* cen = (float*)malloc((size_t)(n_tris > 0 ? n_tris : 1) * 3 * sizeof(float));
    int32_t* q = (int32_t*)malloc((size_t)cap * sizeof(int32_t));
    int32_t* nq = (int32_t*)malloc((size_t)cap * sizeof(int32_t));
    if (!nodes || !cen || !q || !nq) { free(nodes); free(cen); free(q); free(nq); return -3; }
    int64_t nn = 0;
    /* root: initializeLeafEntry(meshBounds.min, meshBounds.max, 0, total) — no pad */
    {
        ubounds rb = ub_setminmax(root_min, root_max);
        float mn[3], mx[3];
        ub_min(&rb, mn);
        ub_max(&rb, mx);
        BVHEntry e;
        e.indexA = 0;
        e.triangleCount = (uint32_t)n_tris;
        e.boundingCornerA.x = mn[0]; e.boundingCornerA.y = mn[1]; e.boundingCornerA.z = mn[2];
        e.boundingCornerB.x = mx[0]; e.boundingCornerB.y = mx[1]; e.boundingCornerB.z = mx[2];
        nodes[nn++] = e;
    }
    /* centroids (v0 + v1 + v2) / 3, BVHGenerator.cs:33-37 */
    for (int64_t i = 0; i < n_tris; i++) {
        const float* a = V + 3 * (int64_t)idx[i * 3];
        const float* b = V + 3 * (int64_t)idx[i * 3 + 1];
        const float* c = V + 3 * (int64_t)idx[i * 3 + 2];
        for (int k = 0; k < 3; k++) cen[i * 3 + k] = ((a[k] + b[k]) + c[k]) / 3.0f;
    }
    int64_t nq_n = 0, q_n = 0;
    q[q_n++] = 0;
    for (int depth = 1; depth <= max_depth; depth++) {
        if (!(q_n > 0)) break;
        for (int64_t qi = 0; qi < q_n; qi++) {
            int32_t ei = q[qi];
            BVHEntry cur = nodes[ei];
            uint32_t first = cur.indexA, cnt = cur.triangleCount;
            float bs[3] = {cur.boundingCornerB.x - cur.boundingCornerA.x, cur.boundingCornerB.y - cur.boundingCornerA.y,
                           cur.boundingCornerB.z - cur.boundingCornerA.z};
            float ca[3] = {cur.boundingCornerA.x, cur.boundingCornerA.y, cur.boundingCornerA.z};
            int axis = bs[0] > bs[1] ? (bs[0] > bs[2] ? 0 : 2) : (bs[1] > bs[2] ? 1 : 2);
            float split = ca[axis] + bs[axis] / 2.0f;
            int64_t i = (int64_t)first, j = i + (int64_t)cnt - 1;
            while (i <= j) {
                if (cen[i * 3 + axis] < split) {
                    i++;
                } else {
                    /* swapEntries(i, j), BVHGenerator.cs:137-152 */
                    for (int k = 0; k < 3; k++) {
                        int32_t ti = idx[i * 3 + k]; idx[i * 3 + k] = idx[j * 3 + k]; idx[j * 3 + k] = ti;
                        float tc = cen[i * 3 + k]; cen[i * 3 + k] = cen[j * 3 + k]; cen[j * 3 + k] = tc;
                    }
                    j--;
                }
            }
            uint32_t ca_n = (uint32_t)i - first, cb_n = cnt - ca_n;
            if (!(ca_n > 0 && cb_n > 0)) continue; /* split failed -> stays a leaf */
            if (cnt <= 5) continue;                 /* maxNodeTriangleCount */
            int32_t ai = (int32_t)nn;
            ubounds ba = calc_bounds(first, ca_n, idx, V);
            BVHEntry ea;
            float mn[3], mx[3];
            ub_min(&ba, mn); ub_max(&ba, mx);
            ea.indexA = first; ea.triangleCount = ca_n;
            ea.boundingCornerA.x = mn[0]; ea.boundingCornerA.y = mn[1]; ea.boundingCornerA.z = mn[2];
            ea.boundingCornerB.x = mx[0]; ea.boundingCornerB.y = mx[1]; ea.boundingCornerB.z = mx[2];
            nodes[nn++] = ea;
            if (ca_n > 2) nq[nq_n++] = ai;
            int32_t bi = (int32_t)nn;
            ubounds bb = calc_bounds((uint32_t)i, cb_n, idx, V);
            BVHEntry eb;
            ub_min(&bb, mn); ub_max(&bb, mx);
            eb.indexA = (uint32_t)i; eb.triangleCount = cb_n;
            eb.boundingCornerA.x = mn[0]; eb.boundingCornerA.y = mn[1]; eb.boundingCornerA.z = mn[2];
            eb.boundingCornerB.x = mx[0]; eb.boundingCornerB.y = mx[1]; eb.boundingCornerB.z = mx[2];
            nodes[nn++] = eb;
            if (cb_n > 2) nq[nq_n++] = bi;
            cur.indexA = (uint32_t)ai;
            cur.triangleCount = 0;
            nodes[ei] = cur;
        }
        memcpy(q, nq, (size_t)nq_n * sizeof(int32_t));
        q_n = nq_n;
        nq_n = 0;
    }
    int64_t ret = nn;
    if (out) {
        if (nn > max_nodes) ret = -(nn + 1);
        else memcpy(out, nodes, (size_t)nn * sizeof(BVHEntry));
    }
    free(nodes); free(cen); free(q); free(nq);
    return ret;
}

/* Exported for tests/test_fmath.py: the number of floats with bit patterns in [lo, hi] on which a fused device
 * form differs (bitwise) from its specification: fn 0 hg_sincosf vs hg_sinf/hg_cosf, 1 hg_acosf_fused vs hg_acosf */
int64_t hgo_fused_mismatches(int32_t fn, uint32_t lo, uint32_t hi) {
    int64_t bad = 0;
    for (uint64_t u = lo; u <= hi; u++) {
        float v, a, b, s, c;
        uint32_t ui = (uint32_t)u, ua, ub;
        memcpy(&v, &ui, 4);
        if (fn == 0) {
            hg_sincosf(v, &s, &c);
            a = hg_sinf(v); b = hg_cosf(v);
            memcpy(&ua, &s, 4); memcpy(&ub, &a, 4);
            if (ua != ub) { bad++; continue; }
            memcpy(&ua, &c, 4); memcpy(&ub, &b, 4);
            if (ua != ub) bad++;
        } else {
            a = hg_acosf_fused(v); b = hg_acosf(v);
            memcpy(&ua, &a, 4); memcpy(&ub, &b, 4);
            if (ua != ub) bad++;
        }
    }
    return bad;
}

/* Exported for tests/test_fmath.py: evaluates the shared arithmetic spec (include/hg_fmath.h) on the host.
 * fn: 0 sin, 1 cos, 2 acos, 3 tan, 4 log, 5 exp, 6 round, 7 rnorm, 8 asin, 9/10 sin/cos of hg_sincosf */
void hgo_fmath(int32_t fn, const float* x, float* y, int64_t n) {
    for (int64_t i = 0; i < n; i++) {
        float v = x[i], r;
        switch (fn) {
            case 0: r = hg_sinf(v); break;
            case 1: r = hg_cosf(v); break;
            case 2: r = hg_acosf(v); break;
            case 3: r = hg_tanf(v); break;
            case 4: r = hg_logf(v); break;
            case 5: r = hg_expf(v); break;
            case 6: r = hg_roundf(v); break;
            case 7: r = hg_rnorm(v); break;
            case 9: { float c; hg_sincosf(v, &r, &c); break; }
            case 10: { float sn; hg_sincosf(v, &sn, &r); break; }
            case 11: r = hg_acosf_fused(v); break;
            default: r = hg_asinf(v); break;
        }
        y[i] = r;
    }
}
