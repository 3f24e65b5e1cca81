// GPU probe (round 4): issue cost of dependent v_mfma_f32_16x16x32_bf16 chains on one wave per SIMD, builtin vs
// inline asm (AGPR A operand, csrc/mlp_rw.hip). Cycles per MFMA from s_memtime around 64 chained products.
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/probes/mfma_chain.hip -o /tmp/mfma_chain
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mv(const u32x4 &a, const u32x4 &b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 ma(const u32x4 &a, const u32x4 &b, f32x4 c)
{
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b));
    return c;
}
__device__ __forceinline__ f32x4 ma6(const u32x4 &a, const u32x4 &b, f32x4 c)
{
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
        : "+v"(c) : "a"(a), "v"(b));
    return c;
}
// two chains interleaved in one statement: A B A B ... (6 products each)
__device__ __forceinline__ void ma2x6(const u32x4 &a, const u32x4 &b0, const u32x4 &b1, f32x4 &c0, f32x4 &c1)
{
    asm("v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\tv_mfma_f32_16x16x32_bf16 %1, %2, %4, %1\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\tv_mfma_f32_16x16x32_bf16 %1, %2, %4, %1\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\tv_mfma_f32_16x16x32_bf16 %1, %2, %4, %1\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\tv_mfma_f32_16x16x32_bf16 %1, %2, %4, %1\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\tv_mfma_f32_16x16x32_bf16 %1, %2, %4, %1\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\tv_mfma_f32_16x16x32_bf16 %1, %2, %4, %1"
        : "+v"(c0), "+v"(c1) : "a"(a), "v"(b0), "v"(b1));
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void k(const u32x4 *w, const u32x4 *x, f32x4 *out, unsigned long long *cyc)
{
    const u32x4 a = w[threadIdx.x], b = x[threadIdx.x], b1 = x[threadIdx.x + 256];
    f32x4 c = {0.f, 0.f, 0.f, 0.f}, c1 = c;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(c), "+v"(c1));
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 64 / (MODE == 2 ? 6 : MODE == 3 ? 6 : 1); ++i) {
        if constexpr (MODE == 0) c = mv(a, b, c);
        else if constexpr (MODE == 1) c = ma(a, b, c);
        else if constexpr (MODE == 2) c = ma6(a, b, c);
        else if constexpr (MODE == 3) ma2x6(a, b, b1, c, c1);
        else if constexpr (MODE == 4) { c = mv(a, b, c); c1 = mv(a, b1, c1); }
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x4 r = c + c1;  // reads the results: the wait for the last MFMA
    asm volatile("" : "+v"(r));
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main()
{
    u32x4 *w, *x;
    f32x4 *o;
    unsigned long long *cy;
    hipMalloc(&w, 256 * 16);
    hipMalloc(&x, 512 * 16);
    hipMalloc(&o, 256 * 256 * 16);
    hipMalloc(&cy, 256 * 8);
    hipMemset(w, 0x3f, 256 * 16);
    hipMemset(x, 0x3f, 512 * 16);
    const char *names[] = {"builtin chain", "asm 1/stmt chain", "asm 6/stmt chain", "asm 2 chains x6/stmt", "builtin 2 chains"};
    const int mfmas[] = {64, 64, 60, 120, 128};
    for (int m = 0; m < 5; ++m) {
        for (int rep = 0; rep < 3; ++rep) {
            switch (m) {
            case 0: hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, w, x, o, cy); break;
            case 1: hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, w, x, o, cy); break;
            case 2: hipLaunchKernelGGL(k<2>, dim3(256), dim3(256), 0, 0, w, x, o, cy); break;
            case 3: hipLaunchKernelGGL(k<3>, dim3(256), dim3(256), 0, 0, w, x, o, cy); break;
            case 4: hipLaunchKernelGGL(k<4>, dim3(256), dim3(256), 0, 0, w, x, o, cy); break;
            }
            hipDeviceSynchronize();
        }
        unsigned long long h[256];
        hipMemcpy(h, cy, sizeof(h), hipMemcpyDeviceToHost);
        unsigned long long mn = h[0];
        for (int i = 0; i < 256; ++i) mn = h[i] < mn ? h[i] : mn;
        printf("%-24s %3d MFMAs: %6llu cycles (min over 256 WGs), %.1f per MFMA\n", names[m], mfmas[m], mn, (double)mn / mfmas[m]);
    }
    return 0;
}
