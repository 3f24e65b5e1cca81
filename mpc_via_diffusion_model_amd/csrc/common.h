// Shared device helpers for the gfx950 kernels of libmpcd.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MPCD_DEV __device__ __forceinline__

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16-byte load through an explicit global (addrspace 1) pointer: global_load_dwordx4, never flat_
// (a flat load also counts on lgkmcnt and forces full drains around LDS waits).
typedef const float __attribute__((address_space(1))) *gptr_f;
MPCD_DEV f32x4 ldg4(const float *p) { return *reinterpret_cast<const f32x4 __attribute__((address_space(1))) *>((gptr_f)p); }

// LDS-only workgroup barrier: retire this wave's LDS traffic, then s_barrier, in ONE asm
// statement so no memory access can be moved across it, and without the vmcnt(0) a
// __syncthreads() fence may add (register-destination global prefetches stay in flight).
MPCD_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Mish(x) = x * tanh(softplus(x)) (torch.nn.Mish). With n = e^x, tanh(log1p(n)) = 1 - 2 / (n(n+2) + 2):
// one v_exp_f32 and one v_rcp_f32 (1 ulp each) plus a multiply, an add, two FMAs and the final product
// (the f32 MFMA and the VALU share issue on gfx950, so every epilogue op counts). Overflow is benign:
// x -> +inf gives n(n+2)+2 = inf, factor 1, Mish(x) = x as in torch; no clamp or select needed.
// Error vs float64 Mish over [-30, 60]: <= 1e-6 absolute everywhere (the 1 - 2r cancellation costs
// relative accuracy only where Mish(x) is ~0, x < -5), 7e-7 relative for |Mish| > 1e-2.
MPCD_DEV float mish(float x)
{
    const float n = __builtin_amdgcn_exp2f(x * 1.44269504088896341f);
    const float r = __builtin_amdgcn_rcpf(__builtin_fmaf(n, n + 2.0f, 2.0f));
    return x * __builtin_fmaf(-2.0f, r, 1.0f);
}

// mish() for the SLP-vectorizable epilogues (csrc/mlp_x3.hip, mlp_sampler.hip, unet_mx.hip): the empty register
// fence on the result keeps each element's Mish in scalar VALU ops. Packed by hipcc's SLP vectorizer (ROCm 7.2)
// such epilogues read v_rcp_f32 results with a v_pk_fma_f32 one wait state later, and a build with that pattern
// gave wrong conv outputs on the GPU (profiles/r3_hazard_ab.txt); tests/test_isa.py keeps every kernel of
// libmpcd.so free of it. The fused U-Net packs its Mish by hand with >= 2 wait states and does not use this.
MPCD_DEV float mish_scalar(float x)
{
    float y = mish(x);
    asm volatile("" : "+v"(y));
    return y;
}

// torch.clamp(x, -1, 1) / torch.clip: a NaN stays NaN (fminf / fmaxf alone would return the bound), so a
// non-finite noise prediction propagates to the samples as in the reference instead of turning into -1.
MPCD_DEV float clamp1(float x)
{
    const float c = fminf(fmaxf(x, -1.0f), 1.0f);
    return x != x ? x : c;
}

// The accurate reference form (expf + IEEE divide), kept for the low-volume prologue kernels.
MPCD_DEV float mish_precise(float x)
{
    const float n = expf(x);
    const float p = n * (n + 2.0f);
    const float r = p / (p + 2.0f);
    return x > 20.0f ? x : x * r;
}

// Philox4x32-10 (Salmon et al., SC'11). counter/key -> 4 uniform uint32.
MPCD_DEV uint4 philox4x32_10(uint4 c, uint2 k)
{
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
        const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += W0;
        k.y += W1;
    }
    return c;
}

// Four standard normals for (seed, candidate, step, element quad) via Box-Muller.
MPCD_DEV f32x4 philox_normal4(uint64_t seed, uint64_t cand, uint32_t step, uint32_t quad)
{
    const uint4 r = philox4x32_10(make_uint4(quad, (uint32_t)cand, (uint32_t)(cand >> 32), step),
                                  make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    const float s = 2.3283064365386963e-10f;  // 2^-32
    const float u0 = ((float)r.x + 1.0f) * s, u1 = (float)r.y * s;
    const float u2 = ((float)r.z + 1.0f) * s, u3 = (float)r.w * s;
    const float ra = __fsqrt_rn(-2.0f * __logf(u0)), rb = __fsqrt_rn(-2.0f * __logf(u2));
    const float ta = 6.2831853071795865f * u1, tb = 6.2831853071795865f * u3;
    // each product in a scalar op (the fence stops SLP packing ra * {cos, sin} into a v_pk_mul_f32 one wait
    // state behind v_sin_f32: the pattern tests/test_isa.py forbids, see mish_scalar)
    float z0 = ra * __cosf(ta), z1 = ra * __sinf(ta), z2 = rb * __cosf(tb), z3 = rb * __sinf(tb);
    asm volatile("" : "+v"(z0), "+v"(z1), "+v"(z2), "+v"(z3));
    return f32x4{z0, z1, z2, z3};
}

// One denoise step of the plan (built on the host from the schedule buffers).
struct StepPlan {
    int32_t t;        // network time index
    int32_t flags;    // bit0: add noise (DDPM t > 0); bit1: final DDIM pair (x <- x0)
    float a, b;       // sqrt_recip_alphas_cumprod[t], sqrt_recipm1_alphas_cumprod[t]
    float c1, c2;     // posterior_mean_coef1/2[t] (DDPM)
    float std;        // sqrt(exp(posterior_log_variance_clipped[t])) (DDPM)
    float sqan, cn;   // sqrt(abar_next), sqrt(1 - abar_next - sigma^2) (DDIM)
    float pad;
};
static_assert(sizeof(StepPlan) == 40, "StepPlan layout");

enum { PLAN_NOISE = 1, PLAN_FINAL = 2 };
enum { MODE_DDPM_CFG = 0, MODE_DDIM_CFG = 1, MODE_DDIM = 2, MODE_EPS = 3, MODE_EPS1 = 4 };
// MODE_EPS / MODE_EPS1: one net forward at plan[0].t on x = noise[0]; eps of the context branch ->
// x_out, of the masked branch -> chain (MODE_EPS, CFG net) or just x_out (MODE_EPS1, 3-arg net).

// One element quad of a denoise step (p_mean_variance_CFG, diffusion_model_base.py:164-178, then
// ddpm_cart_pole_sample_fn, sample_functions.py:17-44; the build-defined CFG-DDIM; the reference's
// ddim_sample, :239-314) in the reference's op order. Every translation unit is compiled with
// -ffp-contract=off, so no product is fused into an add. ec / eu: eps of the context / masked branch
// (eu unused for MODE_DDIM); z: this step's noise (used when the plan adds noise).
MPCD_DEV f32x4 denoise_update4(const StepPlan &sp, int mode, int clamp_x0, float wp1, float wf, const f32x4 &xv,
                               const f32x4 &ec, const f32x4 &eu, const f32x4 &z)
{
    f32x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float xr = xv[r];
        if (mode == MODE_DDPM_CFG) {
            const float x0c = sp.a * xr - sp.b * ec[r];
            const float x0u = sp.a * xr - sp.b * eu[r];
            float x0 = wp1 * x0c - wf * x0u;
            x0 = clamp1(x0);
            const float mean = sp.c1 * x0 + sp.c2 * xr;
            o[r] = (sp.flags & PLAN_NOISE) ? mean + sp.std * z[r] : mean;
        } else if (mode == MODE_DDIM_CFG) {
            float x0 = wp1 * (sp.a * xr - sp.b * ec[r]) - wf * (sp.a * xr - sp.b * eu[r]);
            if (clamp_x0) x0 = clamp1(x0);
            const float e = wp1 * ec[r] - wf * eu[r];
            o[r] = (sp.flags & PLAN_FINAL) ? x0 : x0 * sp.sqan + sp.cn * e;
        } else {
            float x0 = sp.a * xr - sp.b * ec[r];
            if (clamp_x0) x0 = clamp1(x0);
            o[r] = (sp.flags & PLAN_FINAL) ? x0 : x0 * sp.sqan + sp.cn * ec[r];
        }
    }
    return o;
}

// running chain |x| maximum of one element quad (bits of |x| as uint32: a NaN wins the integer max);
// elements are copied to scalars first (a __builtin_bit_cast of a vector-element subscript compiled to
// element 0 for every index)
MPCD_DEV uint32_t absmax_bits4(uint32_t m, const f32x4 &a, const f32x4 &b)
{
    const float ae[4] = {a.x, a.y, a.z, a.w}, be[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t u = __builtin_bit_cast(uint32_t, ae[r]) & 0x7fffffffu;
        const uint32_t v = __builtin_bit_cast(uint32_t, be[r]) & 0x7fffffffu;
        m = max(m, max(u, v));
    }
    return m;
}
