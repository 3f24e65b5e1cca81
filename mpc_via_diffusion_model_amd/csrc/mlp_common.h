// Shared pieces of the two MLP sampler kernels (mlp_sampler.hip: exact-f32 MFMA; mlp_x3.hip:
// fp32-accurate 3-way bf16 split MFMA). Net = build-defined CFG MLP, SURVEY §8a A11.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace mlpc {

constexpr int NLAYER = 14;
constexpr int COND_TOTAL = 448;  // 32+64+128+128+64+32
enum { EPI_NONE = 0, EPI_MISH = 1, EPI_CMISH = 2 };
// CFG-DDPM with caller-supplied noise: its own instantiation, so the in-kernel-Philox variant has no
// global load in the step loop (a conditional noise load made the compiler drain vmcnt(0), i.e. wait
// for the next step's weight prefetch, every step).
constexpr int MODE_DDPM_XN = 16;

template <int D0>
struct Arch {
    static constexpr int K[NLAYER] = {D0, 32, 32, 64, 64, 128, 128, 128, 256, 64, 128, 32, 32, 32};
    static constexpr int N[NLAYER] = {32, 32, 64, 64, 128, 128, 128, 128, 64, 64, 32, 32, 32, D0};
    // Loop form (not recursion) so the device inliner folds every call to a constant.
    __host__ __device__ static constexpr int woff(int l) {  // f32 pack: K*N weights + N biases per layer
        int o = 0;
        for (int i = 0; i < l; ++i) o += K[i] * N[i] + N[i];
        return o;
    }
    static constexpr int total() { return woff(NLAYER); }
    __host__ __device__ static constexpr int woff3(int l) {  // bf16x3 pack, in floats: 3 K*N bf16 + N f32
        int o = 0;
        for (int i = 0; i < l; ++i) o += 3 * K[i] * N[i] / 2 + N[i];
        return o;
    }
    static constexpr int total3() { return woff3(NLAYER); }
    __host__ __device__ static constexpr int boff(int l) {  // biases staged in LDS
        int o = 0;
        for (int i = 0; i < l; ++i) o += N[i];
        return o;
    }
    static constexpr int btotal() { return boff(NLAYER); }
};

// cond block j (0..5) -> column offset in the 448-wide tables
__host__ __device__ constexpr int cond_off(int j) { return j == 0 ? 0 : j == 1 ? 32 : j == 2 ? 96 : j == 3 ? 224 : j == 4 ? 352 : 416; }

// The step plan is read through the constant address space: scalar loads (lgkmcnt), so using it
// never waits on the vector-memory queue that holds the next layers' weight prefetches.
MPCD_DEV StepPlan load_plan(const StepPlan *plan, int s)
{
    typedef const __attribute__((address_space(4))) StepPlan *cplan_t;
    const cplan_t q = (cplan_t)(uintptr_t)plan + s;
    StepPlan r;
    r.t = q->t;
    r.flags = q->flags;
    r.a = q->a;
    r.b = q->b;
    r.c1 = q->c1;
    r.c2 = q->c2;
    r.std = q->std;
    r.sqan = q->sqan;
    r.cn = q->cn;
    r.pad = 0.f;
    return r;
}

// |v| as an ordered integer: max over these bits is max |v| and propagates a NaN (its magnitude bits
// exceed +inf's), which is what the chain clip test needs (mpcd_sample_args.chain_absmax).
MPCD_DEV uint32_t abs_bits(float v) { return __builtin_bit_cast(uint32_t, v) & 0x7fffffffu; }

// Per-candidate chain |x| maximum: each updating lane has folded the x it read and wrote (x_T .. x_0)
// into am[]; reduce them per candidate in LDS (amx[CPW], zeroed at kernel start) and store.
template <int CPW, int THREADS>
MPCD_DEV void store_chain_absmax(uint32_t *amx, const uint32_t (&am)[2], int cl0, int cl1, bool active, float *out,
                                 int64_t cand0, int64_t batch)
{
    if (active) {
        atomicMax(amx + cl0, am[0]);
        if (cl1 >= 0) atomicMax(amx + cl1, am[1]);
    }
    lds_barrier();
    if (threadIdx.x < CPW && cand0 + threadIdx.x < batch)
        out[cand0 + threadIdx.x] = __builtin_bit_cast(float, amx[threadIdx.x]);
}

}  // namespace mlpc
