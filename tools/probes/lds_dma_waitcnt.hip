// CPU-side codegen probe for the MLP sampler's next step: does hipcc (ROCm 7.2, gfx950) keep an
// LDS-DMA weight stream (global_load_lds_dwordx4 into a ring) in flight across unrelated LDS reads, or does it
// wait for the DMA (vmcnt) before every ds_read? Build and inspect:
//   hipcc --offload-arch=gfx950 -O3 -c tools/probes/lds_dma_waitcnt.hip --save-temps -o /tmp/p.o
//   grep -n "s_waitcnt\|global_load_lds\|ds_read\|s_barrier" lds_dma_waitcnt-hip-amdgcn-amd-amdhsa-gfx950.s
// (-DLDS_ONLY_BARRIER: the sampler's fence-free barrier with an explicit vmcnt for the previous slot)
// Findings (round 3): unrelated ds_reads are issued while the DMA is in flight (no wait); __syncthreads() waits
// vmcnt(0), i.e. for the DMA just issued; with the fence-free barrier the compiler still puts vmcnt(0) before the
// read of ring[s & 1] (it cannot tell the dynamic slots apart). probe_two_slots (one __shared__ array per slot,
// loop unrolled by two): the read of slot A while slot B streams has no wait, the read of slot B while slot A
// streams still gets vmcnt(0) — an LDS-DMA weight ring needs its waits checked in the ISA (or explicit
// per-slot objects and a check like tests/test_isa.py) before it is timed.
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void probe(const float *__restrict__ w, const f32x4 *__restrict__ act_in, f32x4 *out,
                                             int steps)
{
    __shared__ f32x4 ring[2][256];   // weight ring (DMA target)
    __shared__ f32x4 act[256];       // activations (ordinary LDS traffic)
    const int t = threadIdx.x;
    act[t] = act_in[t];
    __syncthreads();
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < steps; ++s) {
        // stream the next slot: 16 bytes per lane, straight into LDS
        __builtin_amdgcn_global_load_lds(w + (size_t)(s + 1) * 1024 + t * 4, &ring[(s + 1) & 1][0], 16, 0, 0);
        // unrelated activation reads while the DMA is in flight
        acc += act[(t + s) & 255];
        acc += act[(t * 7 + s) & 255];
        // the slot streamed one iteration ago, after the barrier that publishes it
#ifdef LDS_ONLY_BARRIER
        // the sampler's barrier (no fence): this wave's previous DMA landed (vmcnt(1): only this iteration's is
        // younger), then s_barrier
        asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        acc += ring[s & 1][t ^ 1];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
        __syncthreads();
        acc += ring[s & 1][t ^ 1];
        __syncthreads();
#endif
    }
    out[blockIdx.x * 256 + t] = acc;
}

__global__ __launch_bounds__(256) void probe_two_slots(const float *__restrict__ w, const f32x4 *__restrict__ act_in,
                                                       f32x4 *out, int steps)
{
    __shared__ f32x4 ringA[256], ringB[256], act[256];
    const int t = threadIdx.x;
    act[t] = act_in[t];
    __syncthreads();
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < steps; s += 2) {
        __builtin_amdgcn_global_load_lds(w + (size_t)(s + 1) * 1024 + t * 4, &ringB[0], 16, 0, 0);
        acc += act[(t + s) & 255];
        asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        acc += ringA[t ^ 1];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_global_load_lds(w + (size_t)(s + 2) * 1024 + t * 4, &ringA[0], 16, 0, 0);
        acc += act[(t * 7 + s) & 255];
        asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        acc += ringB[t ^ 1];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    out[blockIdx.x * 256 + t] = acc;
}
