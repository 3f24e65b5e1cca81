// Probe: do f32 MFMAs of one wave and VALU work of another wave on the same SIMD overlap?
// 512-thread workgroups (waves w and w+4 share a SIMD); per wave role: 0 idle, 1 MFMA stream,
// 2 VALU stream (Mish-like: v_exp / v_rcp / fma). Prints ns per launch for each role mix.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int ROLE_LO, int ROLE_HI>
__global__ __launch_bounds__(512, 1) void probe(float *out, int iters)
{
    const int wave = threadIdx.x >> 6;
    const int role = wave < 4 ? ROLE_LO : ROLE_HI;
    float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    float v0 = a, v1 = b, v2 = a + b, v3 = a - b;
    if (role == 1) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, acc1, 0, 0, 0);
                acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, acc2, 0, 0, 0);
                acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, acc3, 0, 0, 0);
            }
        }
    } else if (role == 2) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                // 4 independent chains of (exp, fma, rcp, fma): 2 transcendental + 2 plain per chain
                v0 = __builtin_fmaf(__builtin_amdgcn_rcpf(__builtin_fmaf(__builtin_amdgcn_exp2f(v0), 0.5f, 1.0f)), 0.25f, v0);
                v1 = __builtin_fmaf(__builtin_amdgcn_rcpf(__builtin_fmaf(__builtin_amdgcn_exp2f(v1), 0.5f, 1.0f)), 0.25f, v1);
                v2 = __builtin_fmaf(__builtin_amdgcn_rcpf(__builtin_fmaf(__builtin_amdgcn_exp2f(v2), 0.5f, 1.0f)), 0.25f, v2);
                v3 = __builtin_fmaf(__builtin_amdgcn_rcpf(__builtin_fmaf(__builtin_amdgcn_exp2f(v3), 0.5f, 1.0f)), 0.25f, v3);
            }
        }
    } else if (role == 3) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {  // plain VALU only: 4 independent fma chains x 4
                v0 = __builtin_fmaf(v0, 0.999f, 0.001f); v1 = __builtin_fmaf(v1, 0.999f, 0.001f);
                v2 = __builtin_fmaf(v2, 0.999f, 0.001f); v3 = __builtin_fmaf(v3, 0.999f, 0.001f);
                v0 = __builtin_fmaf(v0, 0.999f, 0.002f); v1 = __builtin_fmaf(v1, 0.999f, 0.002f);
                v2 = __builtin_fmaf(v2, 0.999f, 0.002f); v3 = __builtin_fmaf(v3, 0.999f, 0.002f);
            }
        }
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc0.x + acc1.y + acc2.z + acc3.w + v0 + v1 + v2 + v3;
}

template <int LO, int HI>
float run(float *out, int iters, int blocks)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    probe<LO, HI><<<blocks, 512>>>(out, iters);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) probe<LO, HI><<<blocks, 512>>>(out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main()
{
    const int blocks = 256, iters = 2000;
    float *out;
    hipMalloc(&out, blocks * 512 * sizeof(float));
    // per wave: MFMA role = iters*64 MFMAs (32 cyc each); VALU role = iters*64 chains-steps
    printf("mfma only (waves 0-3)            : %.3f ms\n", run<1, 0>(out, iters, blocks));
    printf("mfma on both waves of a SIMD     : %.3f ms\n", run<1, 1>(out, iters, blocks));
    printf("trans+fma VALU only (waves 0-3)  : %.3f ms\n", run<2, 0>(out, iters, blocks));
    printf("mfma (0-3) + trans VALU (4-7)    : %.3f ms\n", run<1, 2>(out, iters, blocks));
    printf("plain fma VALU only (waves 0-3)  : %.3f ms\n", run<3, 0>(out, iters, blocks));
    printf("mfma (0-3) + plain VALU (4-7)    : %.3f ms\n", run<1, 3>(out, iters, blocks));
    hipFree(out);
    return 0;
}
