// Shared device helpers of the bf16 / f16 matrix-core U-Net kernels (unet_mx.hip: one conv per launch;
// unet_fused.hip: the whole network per workgroup).
//
//  * P = 3 (MPCD_F32X3): every fp32 operand is three bf16 terms (x = x0 + x1 + x2, exact to ~2^-27
//    relative); a dot product accumulates the six partial products whose weight is >= 2^-16 of the
//    leading one, smallest first, in fp32: fp32-level GEMM error at the bf16 rate.
//  * P = 1 (MPCD_F16): fp16 operands, fp32 accumulation.
//  * P = 2 (MPCD_F16X2, the fused U-Net): every operand is two fp16 terms, hi = fp16(x), lo = fp16(x - hi) (the
//    weights scaled per conv by an exact power of two so their lo term stays a normal fp16; the accumulator is
//    unscaled right after the GEMM); a dot product accumulates the three products lo_w hi_x, hi_w lo_x, hi_w hi_x
//    (each dropped or residual term <= 2^-22 of |w||x|): fp32-class error at half the products of P = 3.
#pragma once
#include <hip/hip_runtime.h>

#include "common.h"

namespace mx {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

MPCD_DEV uint32_t pk_bf16(float lo, float hi)
{
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, bf16x2));
}
MPCD_DEV uint32_t pk_f16(float lo, float hi)
{
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, f16x2));
}
MPCD_DEV float bf_lo(uint32_t p) { return __builtin_bit_cast(float, p << 16); }
MPCD_DEV float bf_hi(uint32_t p) { return __builtin_bit_cast(float, p & 0xffff0000u); }

// v - fp32(half H of the packed fp16 pair p), exact (the remainder of a round to nearest), in one v_fma_mix_f32
template <int H>
MPCD_DEV float rem_f16(uint32_t p, float v)
{
    float r;
    if constexpr (H == 0)
        asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(p), "v"(v));
    else
        asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(p), "v"(v));
    return r;
}
// two fp32 -> (hi, lo) fp16 pairs: hi = fp16(a, b), lo = fp16(a - hi, b - hi)
MPCD_DEV void split2_pair(float a, float b, uint32_t &hi, uint32_t &lo)
{
    hi = pk_f16(a, b);
    lo = pk_f16(rem_f16<0>(hi, a), rem_f16<1>(hi, b));
}

// 8 consecutive fp32 -> P planes of 8 values (16 bytes each)
template <int P>
MPCD_DEV void split8(const f32x4 &lo, const f32x4 &hi, u32x4 (&o)[P])
{
    if constexpr (P == 1) {
        o[0] = u32x4{pk_f16(lo.x, lo.y), pk_f16(lo.z, lo.w), pk_f16(hi.x, hi.y), pk_f16(hi.z, hi.w)};
    } else if constexpr (P == 2) {
        uint32_t h[4], l[4];
        split2_pair(lo.x, lo.y, h[0], l[0]);
        split2_pair(lo.z, lo.w, h[1], l[1]);
        split2_pair(hi.x, hi.y, h[2], l[2]);
        split2_pair(hi.z, hi.w, h[3], l[3]);
        o[0] = u32x4{h[0], h[1], h[2], h[3]};
        o[1] = u32x4{l[0], l[1], l[2], l[3]};
    } else {
        const uint32_t a0 = pk_bf16(lo.x, lo.y), a1 = pk_bf16(lo.z, lo.w), a2 = pk_bf16(hi.x, hi.y),
                       a3 = pk_bf16(hi.z, hi.w);
        const f32x4 rl = lo - f32x4{bf_lo(a0), bf_hi(a0), bf_lo(a1), bf_hi(a1)};
        const f32x4 rh = hi - f32x4{bf_lo(a2), bf_hi(a2), bf_lo(a3), bf_hi(a3)};
        const uint32_t b0 = pk_bf16(rl.x, rl.y), b1 = pk_bf16(rl.z, rl.w), b2 = pk_bf16(rh.x, rh.y),
                       b3 = pk_bf16(rh.z, rh.w);
        const f32x4 sl = rl - f32x4{bf_lo(b0), bf_hi(b0), bf_lo(b1), bf_hi(b1)};
        const f32x4 sh = rh - f32x4{bf_lo(b2), bf_hi(b2), bf_lo(b3), bf_hi(b3)};
        o[0] = u32x4{a0, a1, a2, a3};
        o[1] = u32x4{b0, b1, b2, b3};
        o[2] = u32x4{pk_bf16(sl.x, sl.y), pk_bf16(sl.z, sl.w), pk_bf16(sh.x, sh.y), pk_bf16(sh.z, sh.w)};
    }
}

// 4 fp32 -> P planes of 4 values (8 bytes each)
template <int P>
MPCD_DEV void split4(const f32x4 &v, u32x2 (&o)[P])
{
    if constexpr (P == 1) {
        o[0] = u32x2{pk_f16(v.x, v.y), pk_f16(v.z, v.w)};
    } else if constexpr (P == 2) {
        uint32_t h0, l0, h1, l1;
        split2_pair(v.x, v.y, h0, l0);
        split2_pair(v.z, v.w, h1, l1);
        o[0] = u32x2{h0, h1};
        o[1] = u32x2{l0, l1};
    } else {
        const uint32_t a0 = pk_bf16(v.x, v.y), a1 = pk_bf16(v.z, v.w);
        const f32x4 r = v - f32x4{bf_lo(a0), bf_hi(a0), bf_lo(a1), bf_hi(a1)};
        const uint32_t b0 = pk_bf16(r.x, r.y), b1 = pk_bf16(r.z, r.w);
        const f32x4 t = r - f32x4{bf_lo(b0), bf_hi(b0), bf_lo(b1), bf_hi(b1)};
        o[0] = u32x2{a0, a1};
        o[1] = u32x2{b0, b1};
        o[2] = u32x2{pk_bf16(t.x, t.y), pk_bf16(t.z, t.w)};
    }
}

// P planes of 4 values -> 4 fp32 (the split's inverse to within 1 ulp: x0 + x1 + x2 summed large first)
template <int P>
MPCD_DEV f32x4 join4(const u32x2 (&p)[P])
{
    if constexpr (P == 1) {
        return __builtin_convertvector(__builtin_bit_cast(f16x4, p[0]), f32x4);
    } else if constexpr (P == 2) {
        return __builtin_convertvector(__builtin_bit_cast(f16x4, p[0]), f32x4) +
               __builtin_convertvector(__builtin_bit_cast(f16x4, p[1]), f32x4);
    } else {
        f32x4 v = f32x4{bf_lo(p[0].x), bf_hi(p[0].x), bf_lo(p[0].y), bf_hi(p[0].y)};
        v = v + f32x4{bf_lo(p[1].x), bf_hi(p[1].x), bf_lo(p[1].y), bf_hi(p[1].y)};
        return v + f32x4{bf_lo(p[2].x), bf_hi(p[2].x), bf_lo(p[2].y), bf_hi(p[2].y)};
    }
}

template <int P>
MPCD_DEV f32x4 mma(const u32x4 &a, const u32x4 &b, const f32x4 &c)
{
    if constexpr (P == 1 || P == 2)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                      0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                       0, 0, 0);
}

// partial product i of the split: (A plane, B plane), smallest first (P = 2: lo_w hi_x, hi_w lo_x, hi_w hi_x)
constexpr int NPROD(int P) { return P == 1 ? 1 : P == 2 ? 3 : 6; }
template <int P> constexpr int PA(int i)
{
    return P == 1 ? 0 : P == 2 ? (i == 0 ? 1 : 0) : i == 0 ? 2 : i == 1 ? 1 : i == 2 ? 0 : i == 3 ? 1 : 0;
}
template <int P> constexpr int PB(int i)
{
    return P == 1 ? 0 : P == 2 ? (i == 1 ? 1 : 0) : i == 0 ? 0 : i == 1 ? 1 : i == 2 ? 2 : i == 3 ? 0 : i == 4 ? 1 : 0;
}

}  // namespace mx
