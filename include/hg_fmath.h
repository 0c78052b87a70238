/*
 * hg_fmath.h — the fp32 arithmetic SPECIFICATION shared by the HIP megakernel and the CPU oracle.
 *
 * Why this file exists
 * --------------------
 * The reference hot path is HLSL compiled by DXC (`Assets/Scripts/Halogen Shaders/HalgoenCompute.compute:2`,
 * `#pragma use_dxc`).  Its transcendental functions (sin, cos, acos, tan, log, exp) and `normalize`
 * (rsqrt-based) are evaluated by the D3D driver, whose exact bits are unobtainable.  Path tracing turns a
 * 1-ulp difference into a different discrete decision (Russian roulette, refract vs reflect, specular vs
 * diffuse), so "matching within 1e-4" is only achievable if both sides agree bit for bit.
 *
 * This header therefore DEFINES the semantics of every non-IEEE-basic operation the path uses, in terms
 * of IEEE-754 binary32 +, -, *, /, sqrt and exact integer/bit operations only.  Both the gfx950 kernel
 * (hipcc) and the oracle (gcc) compile it with `-ffp-contract=off` and without fast-math, so each call
 * produces identical bits on both sides (gfx950 keeps fp32 denormals by default; x86 SSE does too).
 *
 * The polynomial kernels are the classic Cephes single-precision ones (S. L. Moshier, "Methods and
 * Programs for Mathematical Functions"); their coefficients are published constants.  Accuracy vs libm
 * is checked in tests/test_fmath.py (<= 2 ulp over the domains the path uses).
 *
 * Mapping of HLSL intrinsics used by the reference to this file:
 *   sin/cos  (HalogenRandom.hlsl:288-291,307)       -> hg_sinf / hg_cosf
 *   acos     (HalogenRandom.hlsl:286)               -> hg_acosf
 *   tan      (HalgoenCompute.compute:998)           -> hg_tanf   (= hg_sinf/hg_cosf)
 *   log      (HalogenRandom.hlsl:320)               -> hg_logf
 *   exp      (HalgoenCompute.compute:812)           -> hg_expf
 *   radians  (HalogenDefines.hlsl:12, Random:305)   -> x * HG_DEG2RAD (DXC folds radians() to one fmul)
 *   round    (HalgoenCompute.compute:941)           -> hg_roundf (round-half-to-even, DXIL Round_ne)
 *   min/max  (HalgoenCompute.compute:249-258)       -> fminf/fmaxf (IEEE minNum/maxNum, DXIL FMin/FMax)
 *   normalize                                       -> v * (1/sqrt(dot(v,v)))   (see hg_rnorm)
 *   dot(a,b)                                        -> (a.x*b.x + a.y*b.y) + a.z*b.z, no FMA
 *   lerp(a,b,s)                                     -> a + s*(b - a)
 *
 * This file is C99 and HIP-C++ compatible.  It contains no state.
 */
#ifndef HG_FMATH_H
#define HG_FMATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define HG_FN __host__ __device__ static inline
#else
#define HG_FN static inline
#endif

/* Every translation unit that includes this header must also be compiled with -ffp-contract=off
 * (the Makefiles do); the pragma below additionally pins it for clang/hipcc TUs. */
#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#define HG_INF (__builtin_inff())
#define HG_PI 3.14159265358979323846f
#define HG_DEG2RAD 0.0174532925199432957692f /* float(pi/180) = 0x3C8EFA35, what DXC folds radians() to */

HG_FN uint32_t hg_f2u(float f) {
    union { float f; uint32_t u; } c;
    c.f = f;
    return c.u;
}
HG_FN float hg_u2f(uint32_t u) {
    union { float f; uint32_t u; } c;
    c.u = u;
    return c.f;
}

/* x * 2^n for integer n, exact where the result is representable, IEEE-rounded into the denormal range.
 * Implemented with at most three IEEE multiplies by exact powers of two so both sides round identically. */
HG_FN float hg_ldexpf(float x, int n) {
    if (n > 127) {
        x = x * 1.7014118346046923e38f; /* 2^127 */
        n -= 127;
        if (n > 127) n = 127;
    } else if (n < -126) {
        x = x * 1.1754943508222875e-38f; /* 2^-126 */
        n += 126;
        if (n < -126) {
            x = x * 1.1754943508222875e-38f;
            n += 126;
            if (n < -126) n = -126;
        }
    }
    return x * hg_u2f((uint32_t)(n + 127) << 23);
}

/* round-half-to-even to an integral float (HLSL round -> DXIL Round_ne). */
HG_FN float hg_roundf(float x) {
    float ax = x < 0.0f ? -x : x;
    if (!(ax < 8388608.0f)) return x; /* already integral, or NaN */
    /* adding and subtracting 2^23 rounds to nearest-even in the default rounding mode */
    float r = (ax + 8388608.0f) - 8388608.0f;
    return x < 0.0f ? -r : r;
}

/* ---- sin / cos (Cephes sinf.c / cosf.c, extended-precision Cody-Waite reduction by pi/4) ---- */
#define HG_FOPI 1.27323954473516f
#define HG_DP1 0.78515625f
#define HG_DP2 2.4187564849853515625e-4f
#define HG_DP3 3.77489497744594108e-8f

HG_FN float hg_sincos_poly_(float x, int j, int want_cos) {
    /* x already reduced to [-pi/4, pi/4]; j the octant (0..3) after the sign fold */
    float z = x * x;
    int use_cos = want_cos ? (j == 0 || j == 3) : (j == 1 || j == 2);
    float y;
    if (use_cos) {
        y = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z;
        y = y - 0.5f * z;
        y = y + 1.0f;
    } else {
        y = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * x;
        y = y + x;
    }
    return y;
}

HG_FN float hg_reduce_quadrant_(float ax, int* jout) {
    int j = (int)(ax * HG_FOPI);
    float y;
    if (j & 1) j += 1;
    y = (float)j;
    *jout = j & 7;
    return ((ax - y * HG_DP1) - y * HG_DP2) - y * HG_DP3;
}

HG_FN float hg_sinf(float x) {
    int sign = 1, j;
    float ax = x, r;
    if (x != x) return x;
    if (x < 0.0f) { ax = -x; sign = -1; }
    if (ax == HG_INF) return ax - ax; /* NaN */
    r = hg_reduce_quadrant_(ax, &j); /* j in {0,2,4,6} */
    if (j > 3) { sign = -sign; j -= 4; }
    r = hg_sincos_poly_(r, j, 0);    /* j == 2: sin(x) = cos(x - pi/2) */
    return sign < 0 ? -r : r;
}

HG_FN float hg_cosf(float x) {
    int sign = 1, j;
    float ax = x < 0.0f ? -x : x, r;
    if (x != x) return x;
    if (ax == HG_INF) return ax - ax;
    r = hg_reduce_quadrant_(ax, &j);
    if (j > 3) { j -= 4; sign = -sign; }
    if (j > 1) sign = -sign;
    r = hg_sincos_poly_(r, j, 1);
    return sign < 0 ? -r : r;
}

HG_FN float hg_tanf(float x) { return hg_sinf(x) / hg_cosf(x); }

/* sin and cos of one argument with one reduction and one evaluation of each polynomial: bit-identical to
 * (hg_sinf(x), hg_cosf(x)) for every x (the same operations on the same values; tests/test_fmath.py checks it).
 * The separate forms stay the specification; this is what the device kernels call. */
HG_FN void hg_sincosf(float x, float* s, float* c) {
    float ax = x < 0.0f ? -x : x, r, z, pc, ps;
    int j, flip, ssin, scos;
    if (x != x) { *s = x; *c = x; return; }
    if (ax == HG_INF) { *s = ax - ax; *c = ax - ax; return; }
    r = hg_reduce_quadrant_(ax, &j); /* j in {0,2,4,6} */
    flip = j > 3;
    if (flip) j -= 4;                /* j in {0,2} */
    z = r * r;
    pc = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z;
    pc = pc - 0.5f * z;
    pc = pc + 1.0f;
    ps = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r;
    ps = ps + r;
    ssin = (x < 0.0f) != flip;        /* hg_sinf: sign from x, flipped when j > 3 */
    scos = flip != (j > 1);           /* hg_cosf: flipped when j > 3, and again when j > 1 */
    {
        const float vs = j == 2 ? pc : ps, vc = j == 0 ? pc : ps;
        *s = ssin ? -vs : vs;
        *c = scos ? -vc : vc;
    }
}

/* ---- asin / acos (Cephes asinf.c / acosf.c) ---- */
#define HG_PIO2F 1.5707963267948966192f

HG_FN float hg_asinf(float x) {
    float a = x < 0.0f ? -x : x, z, r;
    int flag = 0;
    if (x != x) return x;
    if (a > 1.0f) return (x - x) / (x - x); /* NaN */
    if (a > 0.5f) {
        z = 0.5f * (1.0f - a);
        r = __builtin_sqrtf(z);
        flag = 1;
    } else {
        r = a;
        z = a * a;
    }
    if (a < 1.0e-4f && !flag) {
        z = a;
    } else {
        z = ((((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z + 7.4953002686e-2f) * z +
             1.6666752422e-1f) * z * r;
        z = z + r;
    }
    if (flag) {
        z = z + z;
        z = HG_PIO2F - z;
    }
    return x < 0.0f ? -z : z;
}

HG_FN float hg_acosf(float x) {
    if (x != x) return x;
    if (x < -0.5f) return HG_PI - 2.0f * hg_asinf(__builtin_sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * hg_asinf(__builtin_sqrtf(0.5f * (1.0f - x)));
    return HG_PIO2F - hg_asinf(x);
}

/* hg_acosf with its three branches sharing one asin evaluation: bit-identical to hg_acosf for every x (each
 * branch's asin argument has |a| <= 0.5 or is NaN, so asin's a > 0.5 path is never taken; tests/test_fmath.py
 * checks every float in [-1, 1]).  Device kernels call this; hg_acosf stays the specification. */
HG_FN float hg_acosf_fused(float x) {
    float a, z, r;
    int lo = x < -0.5f, hi = x > 0.5f;
    if (x != x) return x;
    r = lo ? __builtin_sqrtf(0.5f * (1.0f + x)) : hi ? __builtin_sqrtf(0.5f * (1.0f - x)) : x; /* asin argument */
    /* hg_asinf(r) for |r| <= 0.5 (r >= 0 in the lo / hi branches) */
    if (r != r) {
        z = r;
    } else {
        a = r < 0.0f ? -r : r;
        if (a < 1.0e-4f) {
            z = a;
        } else {
            z = a * a;
            z = ((((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z + 7.4953002686e-2f) * z +
                 1.6666752422e-1f) * z * a;
            z = z + a;
        }
        z = r < 0.0f ? -z : z;
    }
    return lo ? HG_PI - 2.0f * z : hi ? 2.0f * z : HG_PIO2F - z;
}

/* ---- log (Cephes logf.c) ---- */
HG_FN float hg_logf(float x) {
    uint32_t u;
    int e;
    float z, y, fe;
    if (x != x) return x;
    if (x <= 0.0f) return x == 0.0f ? -HG_INF : (x - x) / (x - x);
    if (x == HG_INF) return x;
    u = hg_f2u(x);
    e = 0;
    if ((u >> 23) == 0) { /* denormal: scale up exactly */
        x = x * 16777216.0f; /* 2^24 */
        u = hg_f2u(x);
        e = -24;
    }
    e += (int)(u >> 23) - 126;                 /* frexp exponent */
    x = hg_u2f((u & 0x807fffffu) | 0x3f000000u); /* mantissa in [0.5, 1) */
    if (x < 0.707106781186547524f) {
        e -= 1;
        x = x + x - 1.0f;
    } else {
        x = x - 1.0f;
    }
    z = x * x;
    y = ((((((((7.0376836292e-2f * x - 1.1514610310e-1f) * x + 1.1676998740e-1f) * x - 1.2420140846e-1f) * x +
             1.4249322787e-1f) * x - 1.6668057665e-1f) * x + 2.0000714765e-1f) * x - 2.4999993993e-1f) * x +
         3.3333331174e-1f) * x * z;
    fe = (float)e;
    if (e) y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    z = x + y;
    if (e) z = z + 0.693359375f * fe;
    return z;
}

/* ---- exp (Cephes expf.c) ---- */
HG_FN float hg_expf(float x) {
    float z;
    int n;
    if (x != x) return x;
    if (x > 88.72283905206835f) return HG_INF;
    if (x < -103.278929903431851103f) return 0.0f;
    z = __builtin_floorf(1.44269504088896341f * x + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    n = (int)z;
    z = x * x;
    z = ((((( 1.9875691500e-4f * x + 1.3981999507e-3f) * x + 8.3334519073e-3f) * x + 4.1665795894e-2f) * x +
           1.6666665459e-1f) * x + 5.0000001201e-1f) * z;
    z = z + x;
    z = z + 1.0f;
    return hg_ldexpf(z, n);
}

/* 1/sqrt(d) with IEEE sqrt and IEEE division (the normalize() definition used on both sides). */
HG_FN float hg_rnorm(float d) { return 1.0f / __builtin_sqrtf(d); }

#endif /* HG_FMATH_H */
