// Split-bf16 ("x6") building blocks shared by the conv engine (conv1d.hip) and the fused ResBlock
// kernel (resblock.hip): f32 operands split exactly into bf16 planes, bf16 MFMA, swizzled LDS rows.
#pragma once
#include "rvc_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

RVC_DEV floatx4 mfma_bf16(const uint4& a, const uint4& b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}

RVC_DEV floatx4 mfma_f16(const uint4& a, const uint4& b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8, a), __builtin_bit_cast(halfx8, b), c,
                                                  0, 0, 0);
}

// Split-fp16 arithmetic (RVC_ARITH_F16X3): operands scaled by a power of 2 into fp16's range and split
// exactly into two fp16 pieces v = h + l + r, |r| <= 2^-22 |v| (11 + 11 significant bits); the product
// keeps hH + hL + lH (3 f16 MFMAs, f32 accumulation): ~3 x 2^-22 relative per product, below the f32
// accumulation error of any k-sum longer than ~16 terms.  Weights are scaled per output row at pack time,
// activations per staged tile (its |max|), both undone exactly in the epilogue.
RVC_DEV void split2h(float v, uint32_t& h, uint32_t& l) {
    const _Float16 hh = (_Float16)v;
    const float r = v - (float)hh;  // exact: h is v rounded to 11 significant bits
    const _Float16 ll = (_Float16)r;
    h = __builtin_bit_cast(uint16_t, hh);
    l = __builtin_bit_cast(uint16_t, ll);
}

// exponent E of the power-of-2 scale for values |v| <= amax: amax * 2^E < 2^14 (4x below fp16's 65504)
RVC_DEV int f16_exp(float amax) {
    if (!(amax > 0.f) || !(amax < 3.0e38f)) return 0;
    int e;
    (void)frexpf(amax, &e);  // amax = f 2^e, f in [0.5, 1)
    const int E = 14 - e;
    return E < -100 ? -100 : (E > 100 ? 100 : E);
}

// v -> (h, m, l) bf16 bit patterns, v == h + m + (exactly representable rest), l = bf16(rest)
RVC_DEV void split3(float v, uint32_t& h, uint32_t& m, uint32_t& l) {
    const __bf16 bh = (__bf16)v;
    const float r1 = v - (float)bh;  // exact (Sterbenz)
    const __bf16 bm = (__bf16)r1;
    const float r2 = r1 - (float)bm;  // exact
    const __bf16 bl = (__bf16)r2;
    h = __builtin_bit_cast(uint16_t, bh);
    m = __builtin_bit_cast(uint16_t, bm);
    l = __builtin_bit_cast(uint16_t, bl);
}

// split3 of two values at once: v_cvt_pk_bf16_f32 rounds a pair (round to nearest even, as the scalar
// conversion), the residuals come from the packed halves; h / m / l are the pairs' packed words (element 0 in the
// low half), bit for bit what two split3 calls packed give.
typedef float rvc_f2 __attribute__((ext_vector_type(2)));
typedef float rvc_f2u __attribute__((ext_vector_type(2), aligned(4)));  // a float pair at any float offset
typedef __bf16 rvc_bf2 __attribute__((ext_vector_type(2)));
RVC_DEV uint32_t pk_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((rvc_f2){a, b}, rvc_bf2));
}
RVC_DEV void split3_pk(float v0, float v1, uint32_t& h, uint32_t& m, uint32_t& l) {
    h = pk_bf16(v0, v1);
    const float r0 = v0 - __uint_as_float(h << 16), r1 = v1 - __uint_as_float(h & 0xffff0000u);
    m = pk_bf16(r0, r1);
    const float s0 = r0 - __uint_as_float(m << 16), s1 = r1 - __uint_as_float(m & 0xffff0000u);
    l = pk_bf16(s0, s1);
}

// split2h of two values at once (v_cvt_pk_f16_f32 rounds a pair to nearest even, as the scalar conversion): h / l
// are the packed words, element 0 in the low half -- bit for bit two split2h calls packed.
typedef _Float16 rvc_h2 __attribute__((ext_vector_type(2)));
RVC_DEV uint32_t pk_f16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((rvc_f2){a, b}, rvc_h2));
}
RVC_DEV void split2h_pk(float v0, float v1, uint32_t& h, uint32_t& l) {
    h = pk_f16(v0, v1);
    const rvc_h2 hh = __builtin_bit_cast(rvc_h2, h);
    l = pk_f16(v0 - (float)hh.x, v1 - (float)hh.y);
}

// NP = MFMA passes per product: 6 (f32-accurate, above), 3 (hH + hM + mH: 16-bit-mantissa products,
// ~2^-16 relative) or 1 (hH: plain bf16 operands, f32 accumulation).  Only the NPL = 3 / 2 / 1 planes a
// pass set reads are staged and loaded.  LDS rows are [pos][NPL planes][4 x 16 B]; the 16-B group is
// XOR-swizzled so that a ds_read_b128 of B operands (lane l: position base + (l & 15), group l >> 4) is
// conflict-free under gfx950's lane grouping for 16-B reads -- {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}
// and the same +32 (MI355X_MICROARCH.md, LDS): each group holds 4 lanes per position residue mod 4 at
// 4 distinct (position >> 1) & 3, so NPL 3 and 1 swizzle by (pos >> 1) & 3 within the plane and NPL 2
// by pos & 7 across the two planes (4 LDS cycles per read instead of 7-8 with a (pos >> 2) swizzle; the
// loaders' 8-lane ds_write_b128 groups stay at <= 2 positions per bank quad).
template <int NPL>
RVC_DEV int x_slot(int pos, int q, int g) {
    if constexpr (NPL == 2) return pos * 8 + ((4 * q + g) ^ (pos & 7));
    else return pos * (4 * NPL) + 4 * q + (g ^ ((pos >> 1) & 3));
}

