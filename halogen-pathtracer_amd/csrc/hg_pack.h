// hg_pack.h — the display formats of hg_readback_begin_format (include/halogen_abi.h), one definition for the device
// untile kernel (hg_runtime.hip) and the host packer hg_pack_display.
//
// The reference blits its accumulation target into the URP camera colour target (HalogenRenderPass.cs:345), which
// Assets/Settings/URP-HighFidelity.asset:26-27 configures as an HDR target of m_HDRColorBufferPrecision 0: the 32-bit
// packed float format R11G11B10 (DXGI_FORMAT_R11G11B10_FLOAT: R in bits 0-10, G in 11-21, B in 22-31; alpha dropped).
// Our conversion rules (integer arithmetic, identical on host and device; D3D's own converter is not available here,
// so parity with it is UNPINNED):
//   - R and G: unsigned float, 5-bit exponent (bias 15), 6-bit mantissa; B: 5-bit exponent, 5-bit mantissa;
//   - round to nearest, ties to even, including into the denormal range (exponent field 0);
//   - a finite value that rounds past the largest finite (65,024 for R/G, 64,512 for B) becomes +Inf, as does +Inf;
//   - negative values (-0 and -Inf included) and NaN become 0.
// RGBA16F: IEEE binary16 per channel (alpha kept), round to nearest even, overflow to +/-Inf, signs kept, NaN -> the
// quiet NaN 0x7E00.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define HG_PACK_FN __host__ __device__ __forceinline__
#else
#define HG_PACK_FN static inline
#endif

// A non-negative float (bits u: sign 0, not NaN / Inf) rounded to an unsigned float of `mbits` mantissa bits and a
// 5-bit exponent of bias 15: the (exponent << mbits | mantissa) field; 31 << mbits (Inf) on overflow.
HG_PACK_FN uint32_t hg_pack_ufloat5(uint32_t u, uint32_t mbits) {
    const uint32_t ef = u >> 23;  // the float's exponent field
    if (ef == 0u) return 0u;      // zero or a float32 denormal: far below half of the smallest target denormal
    const uint32_t sig = 0x800000u | (u & 0x7FFFFFu);
    const int32_t e = int32_t(ef) - 127;  // value = sig * 2^(e - 23)
    uint32_t v, rem, half;
    if (e >= -14) {  // normal target: exponent field e + 15, mantissa = top mbits bits of the 23
        if (e > 15) return 31u << mbits;
        const uint32_t sh = 23u - mbits;
        v = (uint32_t(e + 15) << mbits) | ((sig & 0x7FFFFFu) >> sh);
        rem = sig & ((1u << sh) - 1u);
        half = 1u << (sh - 1u);
    } else {  // denormal target: units of 2^(-14 - mbits); value / unit = sig >> (9 - mbits - e)
        const uint32_t sh = uint32_t(9 - int32_t(mbits) - e);  // >= 24 - mbits
        if (sh > 24u) return 0u;                               // below half a unit
        v = sig >> sh;
        rem = sig & ((1u << sh) - 1u);
        half = 1u << (sh - 1u);
    }
    if (rem > half || (rem == half && (v & 1u))) ++v;  // a carry moves into the exponent field (exact)
    return v >= (31u << mbits) ? (31u << mbits) : v;
}

HG_PACK_FN uint32_t hg_pack_uf(float x, uint32_t mbits) {
    union {
        float f;
        uint32_t u;
    } b;
    b.f = x;
    if (b.u >= 0x7F800001u) return 0u;                   // NaN (positive) or any negative value, -0 and -NaN included
    if (b.u == 0x7F800000u) return 31u << mbits;         // +Inf
    return hg_pack_ufloat5(b.u, mbits);
}

HG_PACK_FN uint32_t hg_pack_r11g11b10(float r, float g, float b) {
    return hg_pack_uf(r, 6u) | (hg_pack_uf(g, 6u) << 11) | (hg_pack_uf(b, 5u) << 22);
}

HG_PACK_FN uint32_t hg_pack_half(float x) {
    union {
        float f;
        uint32_t u;
    } b;
    b.f = x;
    const uint32_t sign = (b.u >> 16) & 0x8000u, mag = b.u & 0x7FFFFFFFu;
    if (mag > 0x7F800000u) return 0x7E00u;              // NaN
    if (mag == 0x7F800000u) return sign | 0x7C00u;      // +/-Inf
    return sign | hg_pack_ufloat5(mag, 10u);            // 10-bit mantissa, overflow -> Inf
}

// 4 halves as two words, channel 0 in the low half of the first word (the memory order of an RGBA16F texel)
HG_PACK_FN void hg_pack_rgba16f(float r, float g, float b, float a, uint32_t out[2]) {
    out[0] = hg_pack_half(r) | (hg_pack_half(g) << 16);
    out[1] = hg_pack_half(b) | (hg_pack_half(a) << 16);
}
