// Candidate rollout + MPC cost + selection, fp64, one thread per candidate.
//
// Per candidate: u = LimitsNormalizer.unnormalize(u_norm) in fp32 (normalization.py:156-167, with
// the GLOBAL clip rule computed by clip_flag_kernel), cast exactly to fp64, then the system's
// Euler / ZOH rollout and the MPC objective in fp64 with the reference's left-to-right operation
// order (built with -ffp-contract=off, so no contraction changes a rounding).
// Coalescing: a workgroup stages its candidates' [H][n_u] rows through LDS with contiguous
// loads; each thread then walks its own row from LDS.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "../../include/mpcd.h"
#include "internal.h"

namespace {

constexpr int RT_THREADS = 64;  // candidates per workgroup (one wave: the fused argmin is a wave reduction)
static_assert(RT_THREADS == kRolloutBlock, "RolloutSelect partial count");

struct SysK {
    int32_t system, cost_kind, nx, nu;
    double params[24];
    double Q[12], R[4], P[12], xr[12];
    double x0[12];
    float umin[4], umax[4];
};

struct MinMax {
    float mn[16], mx[16];
};

// Fused selection (single-rank control step): block argmins -> the last block reduces them, writes
// *best and the winner's unnormalised [H][n_u] row. part_* hold one entry per block; counter is zero
// between launches (the last block resets it).
struct SelectK {
    mpcd_best *best;
    float *row_out;      // [H * n_u] unnormalised winner row
    double *part_cost;   // [gridDim.x]
    int64_t *part_idx;   // [gridDim.x]
    unsigned *counter;
    int64_t offset;      // global index of candidate 0
    int32_t *code_out;   // optional: flags[0] copied next to the winner (saves the caller a device copy)
    const float *clip_src;  // optional: the clip code computed here over clip_src[0, clip_n) (RolloutSelect)
    int64_t clip_n;
    char *host_out;         // optional: the result block mirrored to mapped host memory + a completion word
    uint32_t *host_flag;
    uint32_t host_seq;
};

// (v, i) beats (bv, bi): NaN = +inf, lower cost, then lower index; i < 0 = empty
__device__ __forceinline__ bool better(double v, int64_t i, double bv, int64_t bi)
{
    return i >= 0 && (bi < 0 || v < bv || (v == bv && i < bi));
}
__device__ __forceinline__ void wave_argmin(double &v, int64_t &i)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const double ov = __shfl_xor(v, m);
        const int64_t oi = __shfl_xor(i, m);
        if (better(ov, oi, v, i)) { v = ov; i = oi; }
    }
}

// State / input sizes per system: compile-time, so every per-candidate array lives in registers
// (a runtime n_x indexed them dynamically and put them in scratch memory).
template <int SYS> struct SysDim;
template <> struct SysDim<MPCD_SYS_CARTPOLE_LIN5> { static constexpr int NX = 5, NU = 1; };
template <> struct SysDim<MPCD_SYS_CARTPOLE_NL5> { static constexpr int NX = 5, NU = 1; };
template <> struct SysDim<MPCD_SYS_CARTPOLE_ZOH4> { static constexpr int NX = 4, NU = 1; };
template <> struct SysDim<MPCD_SYS_DOUBLE_INT2D> { static constexpr int NX = 4, NU = 2; };
template <> struct SysDim<MPCD_SYS_PENDULUM> { static constexpr int NX = 2, NU = 1; };
template <> struct SysDim<MPCD_SYS_QUADROTOR12> { static constexpr int NX = 12, NU = 4; };

template <int N>
__device__ __forceinline__ double quadform(const double *w, const double *x, const double *ref)
{
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const double e = x[j] - ref[j];
        s = s + w[j] * (e * e);
    }
    return s;
}

// x_{k+1} = f(x_k, u_k). Parameter layouts are filled by mpc_via_diffusion_model_amd/systems.py.
template <int SYS>
__device__ __forceinline__ void dyn_step(const SysK &S, const double *x, const double *u, double *xn)
{
    const double *p = S.params;
    switch (SYS) {
    case MPCD_SYS_CARTPOLE_LIN5: {
        // EulerForwardCartpole_virtual, xdot_new (Cart_Diffusion_inference.py:183-197)
        // p: dt, -k*v2, (lm^2)*G*v2/il, lm*c*v2/il, v2, -l*m*k*v1/(M+m), lm*G*v1, c*v1, lm*v1/(M+m), 2/pi, pi
        double xd[5];
        xd[0] = x[1];
        xd[1] = p[1] * x[1] + p[2] * x[2] - p[3] * x[3] + p[4] * u[0];
        xd[2] = x[3];
        xd[3] = p[5] * x[1] + p[6] * x[2] - p[7] * x[3] + p[8] * u[0];
        xd[4] = -p[9] * (x[2] - p[10]) * x[3];
        for (int i = 0; i < 5; ++i) xn[i] = x[i] + xd[i] * p[0];
        break;
    }
    case MPCD_SYS_CARTPOLE_NL5: {
        // nmpc_multi_process_collect_data.py:121-137. p: dt, MPLP, MPG, M_TOTAL, M_POLE, MTG, MTLP, 2/pi, pi
        const double s = sin(x[2]), c = cos(x[2]);
        const double dd = p[3] - p[4] * c;
        double xd[5];
        xd[0] = x[1];
        xd[1] = (p[1] * -s * (x[3] * x[3]) + p[2] * s * c + u[0]) / (dd * dd);
        xd[2] = x[3];
        xd[3] = (-p[1] * s * c * (x[3] * x[3]) - p[5] * s - c * u[0]) / (p[6] - p[1] * (c * c));
        xd[4] = -p[7] * (x[2] - p[8]) * x[3];
        for (int i = 0; i < 5; ++i) xn[i] = x[i] + xd[i] * p[0];
        break;
    }
    case MPCD_SYS_CARTPOLE_ZOH4:
        // Diffusion_MPC_Inference.py:74-82. p: A_d row-major [16], B_d [4]
        for (int i = 0; i < 4; ++i)
            xn[i] = p[4 * i] * x[0] + p[4 * i + 1] * x[1] + p[4 * i + 2] * x[2] + p[4 * i + 3] * x[3] + p[16 + i] * u[0];
        break;
    case MPCD_SYS_DOUBLE_INT2D:
        // p: dt, 0.5*dt*dt
        xn[0] = x[0] + p[0] * x[2] + p[1] * u[0];
        xn[1] = x[1] + p[0] * x[3] + p[1] * u[1];
        xn[2] = x[2] + p[0] * u[0];
        xn[3] = x[3] + p[0] * u[1];
        break;
    case MPCD_SYS_PENDULUM:
        // p: dt, g/l, damping, 1/(m l^2)
        xn[0] = x[0] + p[0] * x[1];
        xn[1] = x[1] + p[0] * (-p[1] * sin(x[0]) - p[2] * x[1] + p[3] * u[0]);
        break;
    case MPCD_SYS_QUADROTOR12: {
        // p: dt, m, g, Ix, Iy, Iz
        const double sph = sin(x[3]), cph = cos(x[3]), sth = sin(x[4]), cth = cos(x[4]);
        const double sps = sin(x[5]), cps = cos(x[5]);
        const double f_m = (p[1] * p[2] + u[0]) / p[1];
        double xd[12];
        xd[0] = x[6];
        xd[1] = x[7];
        xd[2] = x[8];
        xd[3] = x[9] + (x[10] * sph + x[11] * cph) * (sth / cth);
        xd[4] = x[10] * cph - x[11] * sph;
        xd[5] = (x[10] * sph + x[11] * cph) / cth;
        xd[6] = f_m * (cph * sth * cps + sph * sps);
        xd[7] = f_m * (cph * sth * sps - sph * cps);
        xd[8] = f_m * (cph * cth) - p[2];
        xd[9] = ((p[4] - p[5]) * x[10] * x[11] + u[1]) / p[3];
        xd[10] = ((p[5] - p[3]) * x[9] * x[11] + u[2]) / p[4];
        xd[11] = ((p[3] - p[4]) * x[9] * x[10] + u[3]) / p[5];
        for (int i = 0; i < 12; ++i) xn[i] = x[i] + p[0] * xd[i];
        break;
    }
    }
}

// LimitsNormalizer's global clip test x.max() > 1+eps or x.min() < -1-eps (normalization.py:160) with
// torch's NaN semantics: a NaN makes max() and min() NaN, both comparisons false, no clip. Result code:
// 0 = in range, 1 = clip, 2 = a NaN was seen (no clip; 2 also wins a max-reduction over ranks, as a NaN
// on any rank makes the global max NaN). Consumers clip iff the flag is exactly 1.
// One launch, no memset: blocks OR bit0 (out of range) / bit1 (NaN) into ws[0]; the last block to finish
// (ws[1] counts them) moves the result to *flag and leaves ws zeroed for the next launch on the stream.
__device__ __forceinline__ unsigned clip_bits(float v, float hi, float lo)
{
    return ((v > hi) | (v < lo)) ? 1u : (v != v ? 2u : 0u);
}
__device__ __forceinline__ int clip_code(unsigned bits) { return (bits & 2u) ? 2 : (int)(bits & 1u); }

__global__ __launch_bounds__(256) void clip_flag_kernel(const float *x, int64_t n, int *flag, unsigned *ws)
{
    const float hi = (float)(1.0 + 1e-4), lo = (float)(-1.0 - 1e-4);
    unsigned any = 0;
    const int64_t n4 = ((uintptr_t)x & 15) ? 0 : n >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const f32x4 v = reinterpret_cast<const f32x4 *>(x)[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) any |= clip_bits(v[e], hi, lo);
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        any |= clip_bits(x[i], hi, lo);
    __shared__ unsigned blk;
    if (threadIdx.x == 0) blk = 0;
    __syncthreads();
    if (any) atomicOr(&blk, any);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (blk) atomicOr(ws, blk);
        __threadfence();
        if (atomicAdd(ws + 1, 1u) == gridDim.x - 1) {
            __threadfence();
            *flag = clip_code(atomicExch(ws, 0u));
            atomicExch(ws + 1, 0u);
        }
    }
}

__device__ __forceinline__ float unnorm1(float v, bool clip, float mn, float mx)
{
    if (clip) v = clamp1(v);
    const float h = (v + 1.0f) / 2.0f;
    return h * (mx - mn) + mn;
}

__global__ void unnormalize_kernel(const float *x, int64_t n, int dim, const int *flag, const MinMax lim, float *out)
{
    const bool clip = *flag == 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % dim);
        out[i] = unnorm1(x[i], clip, lim.mn[c], lim.mx[c]);
    }
}

// x0_dev == nullptr: every candidate starts from S.x0; else candidate b starts from x0_dev[b / group]
// (closed loop: one plant state per group of candidates). flags[b / group] is that group's clip flag
// (group = batch for the single-state case: one global flag).
// SEL: also select (SelectK above) - one launch for rollout, cost, argmin and the winner's row.
template <int SYS, bool SEL>
__global__ __launch_bounds__(RT_THREADS) void rollout_cost_kernel(const SysK S, const float *u_norm, const int *flags,
                                                                  const double *x0_dev, int64_t group, int64_t batch,
                                                                  int H, double *cost, const SelectK K)
{
    constexpr int nx = SysDim<SYS>::NX, nu = SysDim<SYS>::NU;
    extern __shared__ float su[];  // [RT_THREADS][H*nu + 1]
    const int row = H * nu, stride = row + 1;
    const int64_t c0 = (int64_t)blockIdx.x * RT_THREADS;
    const int64_t nvalid = min((int64_t)RT_THREADS, batch - c0);
    const float *src = u_norm + (size_t)c0 * row;
    if ((row & 3) == 0) {  // 16-byte loads (a row never straddles a quad)
        // in batches of UNR loads per lane, all issued before the first LDS store: one memory latency per batch
        // (a load -> store loop waits for every load in turn: 16 latencies at H = 32, nu = 2)
        constexpr int UNR = 8;
        const int nq = (int)(nvalid * row / 4);
        for (int base = 0; base < nq; base += UNR * RT_THREADS) {
            f32x4 v[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int i = base + u * RT_THREADS + (int)threadIdx.x;
                v[u] = i < nq ? ldg4(src + 4 * i) : f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int i = base + u * RT_THREADS + (int)threadIdx.x;
                if (i < nq) {
                    const int c = 4 * i / row, k = 4 * i - c * row;
#pragma unroll
                    for (int e = 0; e < 4; ++e) su[c * stride + k + e] = v[u][e];
                }
            }
        }
    } else {
        for (int i = threadIdx.x; i < nvalid * row; i += RT_THREADS) {
            const int c = i / row, k = i - c * row;
            su[c * stride + k] = src[i];
        }
    }
    int code = 0;  // SEL with clip_src: the clip code, recomputed by every workgroup (clip_flag_kernel's test)
    if constexpr (SEL) {
        if (K.clip_src) {
            const float hi = (float)(1.0 + 1e-4), lo = (float)(-1.0 - 1e-4);
            unsigned any = 0;
            const int64_t n4 = ((uintptr_t)K.clip_src & 15) ? 0 : K.clip_n >> 2;
#pragma unroll 8
            for (int64_t i = threadIdx.x; i < n4; i += RT_THREADS) {  // unrolled: eight loads in flight per lane
                const f32x4 v = ldg4(K.clip_src + 4 * i);
#pragma unroll
                for (int e = 0; e < 4; ++e) any |= clip_bits(v[e], hi, lo);
            }
            for (int64_t i = 4 * n4 + threadIdx.x; i < K.clip_n; i += RT_THREADS) any |= clip_bits(K.clip_src[i], hi, lo);
            __shared__ unsigned blk;
            if (threadIdx.x == 0) blk = 0;
            __syncthreads();
            if (any) atomicOr(&blk, any);
            __syncthreads();
            code = clip_code(blk);
        }
    }
    __syncthreads();
    const int64_t b = min(c0 + threadIdx.x, batch - 1);  // lanes past the batch recompute the last one
    const bool clip = (SEL && K.clip_src) ? code == 1 : flags[b / group] == 1;
    float mn[nu], mx[nu];
#pragma unroll
    for (int i = 0; i < nu; ++i) { mn[i] = S.umin[i]; mx[i] = S.umax[i]; }
    const float *ur = su + (b - c0) * stride;
    double x[nx], xn[nx], u[nu];
#pragma unroll
    for (int i = 0; i < nx; ++i) x[i] = x0_dev ? x0_dev[(b / group) * nx + i] : S.x0[i];
    double J;
    if (S.cost_kind == MPCD_COST_CALMPC) {
        // calMPCCost (Cart_Diffusion_inference.py:247-283); num_u = 1 (batch axis of u_hor)
        J = 0.0;
        for (int i = 0; i < nx; ++i) J = J + S.Q[i] * (x[i] * x[i]);
        u[0] = (double)unnorm1(ur[0], clip, mn[0], mx[0]);
        J = J + S.R[0] * (u[0] * u[0]);
        for (int i = 0; i < nx; ++i) xn[i] = x[i];
        double ucur = u[0];
        for (int i = 1; i < H - 1; ++i) {
            dyn_step<SYS>(S, x, &ucur, xn);
            const double un = (double)unnorm1(ur[i * nu], clip, mn[0], mx[0]);
            for (int j = 1; j < nx; ++j) J = J + S.Q[j] * (xn[j] * xn[j]);
            J = J + S.R[0] * (un * un);
            ucur = un;
            for (int j = 0; j < nx; ++j) x[j] = xn[j];
        }
        for (int i = 0; i < nx; ++i) J = J + S.P[i] * (xn[i] * xn[i]);
    } else {
        const double zero[4] = {0.0, 0.0, 0.0, 0.0};
        J = quadform<nx>(S.Q, x, S.xr);
        for (int k = 0; k < H; ++k) {
            for (int i = 0; i < nu; ++i) u[i] = (double)unnorm1(ur[k * nu + i], clip, mn[i], mx[i]);
            dyn_step<SYS>(S, x, u, xn);
            const double sx = k < H - 1 ? quadform<nx>(S.Q, xn, S.xr) : quadform<nx>(S.P, xn, S.xr);
            const double sv = quadform<nu>(S.R, u, zero);
            J = J + (sx + sv);
            for (int j = 0; j < nx; ++j) x[j] = xn[j];
        }
    }
    if (c0 + threadIdx.x < batch) cost[b] = J;
    if constexpr (SEL) {
        double v = isnan(J) ? INFINITY : J;
        int64_t i = c0 + threadIdx.x < batch ? b : -1;
        wave_argmin(v, i);  // RT_THREADS == one wave
        __shared__ bool last;
        if (threadIdx.x == 0) {
            K.part_cost[blockIdx.x] = v;
            K.part_idx[blockIdx.x] = i;
            __threadfence();
            last = atomicAdd(K.counter, 1u) == gridDim.x - 1;
        }
        __syncthreads();
        if (!last) return;
        __threadfence();
        v = INFINITY;
        i = -1;
        for (int k = threadIdx.x; k < (int)gridDim.x; k += RT_THREADS) {
            const double pv = __builtin_nontemporal_load(K.part_cost + k);
            const int64_t pi = __builtin_nontemporal_load(K.part_idx + k);
            if (better(pv, pi, v, i)) { v = pv; i = pi; }
        }
        wave_argmin(v, i);
        const int32_t ccode = K.clip_src ? code : flags[0];
        float *hrow = K.host_out ? reinterpret_cast<float *>(K.host_out + sizeof(mpcd_best)) : nullptr;
        if (threadIdx.x == 0) {
            const mpcd_best bst{v, i < 0 ? -1 : K.offset + i};
            *K.best = bst;
            *K.counter = 0u;
            if (K.code_out) *K.code_out = ccode;
            if (hrow) {
                *reinterpret_cast<mpcd_best *>(K.host_out) = bst;
                *reinterpret_cast<int32_t *>(hrow + row) = ccode;
            }
        }
        if (i >= 0 && K.row_out) {
            const bool clip0 = K.clip_src ? code == 1 : flags[0] == 1;
            for (int k = threadIdx.x; k < row; k += RT_THREADS) {
                const float o = unnorm1(u_norm[(size_t)i * row + k], clip0, S.umin[k % nu], S.umax[k % nu]);
                K.row_out[k] = o;
                if (hrow) hrow[k] = o;
            }
        }
        if (hrow) {  // every lane's host stores ordered before the completion word
            __threadfence_system();
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_store(K.host_flag, K.host_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Per-group clip flags: flags[g] = the clip code above over x[g*group_elems, (g+1)*group_elems)
// (LimitsNormalizer's rule applied to each plant state's own candidate batch). One workgroup per group:
// every flag is written, so no memset is needed.
__global__ __launch_bounds__(256) void clip_flags_kernel(const float *x, int64_t group_elems, int *flags)
{
    const float hi = (float)(1.0 + 1e-4), lo = (float)(-1.0 - 1e-4);
    const float *g = x + (size_t)blockIdx.x * group_elems;
    unsigned any = 0;
    for (int64_t i = threadIdx.x; i < group_elems; i += blockDim.x) any |= clip_bits(g[i], hi, lo);
    __shared__ unsigned blk;
    if (threadIdx.x == 0) blk = 0;
    __syncthreads();
    if (any) atomicOr(&blk, any);
    __syncthreads();
    if (threadIdx.x == 0) flags[blockIdx.x] = clip_code(blk);
}

// normalize_condition for a batch of plant states (normalization.py:149-154 in fp64, then the net's
// .float()): ctx[m][c] = fp32(2 * ((x[m][c] - min[c]) / den[c]) - 1), den = fp32(max - min).
struct NormK {
    double mn[16], den[16];
};
__global__ void normalize_states_kernel(const double *x, int64_t M, int C, const NormK nk, float *out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * C) return;
    const int c = (int)(i % C);
    out[i] = (float)(2.0 * ((x[i] - nk.mn[c]) / nk.den[c]) - 1.0);
}

// One closed-loop control step per plant state m (one workgroup each): the candidate of its group
// [m*group, (m+1)*group) with the lowest cost (NaN = +inf, lowest index on ties; or the group's first
// candidate, the reference scripts' n_samples = 1 convention), its u[0] unnormalised with the
// group's clip flag and rounded to `decimals` places (the reference's round(u, 4) on the fp32 value
// promoted to double; < 0: none), then the plant step x[m] <- f(x[m], u0) in fp64.
constexpr int CS_THREADS = 256;
template <int SYS>
__global__ __launch_bounds__(CS_THREADS) void control_step_kernel(const SysK S, double *x_dev, int64_t group,
                                                                  const float *u_norm, int H, const double *cost,
                                                                  const int *flags, int select_first, int decimals,
                                                                  double *u_applied, int64_t *best_idx, double *best_cost)
{
    constexpr int nx = SysDim<SYS>::NX, nu = SysDim<SYS>::NU;
    __shared__ double sv[CS_THREADS];
    __shared__ int64_t si[CS_THREADS];
    const int64_t m = blockIdx.x, base = m * group;
    double bv = INFINITY;
    int64_t bi = -1;
    if (select_first) {
        if (threadIdx.x == 0) {
            bi = base;
            bv = cost[base];
        }
    } else {
        for (int64_t i = threadIdx.x; i < group; i += CS_THREADS) {
            double v = cost[base + i];
            if (isnan(v)) v = INFINITY;
            if (bi < 0 || v < bv) {
                bv = v;
                bi = base + i;
            }
        }
    }
    sv[threadIdx.x] = bv;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int w = CS_THREADS / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const double ov = sv[threadIdx.x + w];
            const int64_t oi = si[threadIdx.x + w];
            const double mv = sv[threadIdx.x];
            const int64_t mi = si[threadIdx.x];
            if (oi >= 0 && (mi < 0 || ov < mv || (ov == mv && oi < mi))) {
                sv[threadIdx.x] = ov;
                si[threadIdx.x] = oi;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const int64_t idx = si[0];
    const bool clip = flags[m] == 1;
    double x[nx], xn[nx], u[nu];
#pragma unroll
    for (int i = 0; i < nx; ++i) x[i] = x_dev[m * nx + i];
#pragma unroll
    for (int i = 0; i < nu; ++i) {
        double v = (double)unnorm1(u_norm[(size_t)idx * H * nu + i], clip, S.umin[i], S.umax[i]);
        if (decimals >= 0) {
            const double sc = pow(10.0, (double)decimals);
            v = rint(v * sc) / sc;
        }
        u[i] = v;
    }
    dyn_step<SYS>(S, x, u, xn);
#pragma unroll
    for (int i = 0; i < nx; ++i) x_dev[m * nx + i] = xn[i];
#pragma unroll
    for (int i = 0; i < nu; ++i) u_applied[m * nu + i] = u[i];
    best_idx[m] = idx;
    best_cost[m] = cost[idx];
}

// Single-workgroup argmin: NaN -> +inf; ties -> lowest index.
__global__ __launch_bounds__(1024) void argmin_kernel(const double *cost, int64_t n, int64_t offset, mpcd_best *best)
{
    __shared__ double sv[1024];
    __shared__ int64_t si[1024];
    double bv = INFINITY;
    int64_t bi = -1;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        double v = cost[i];
        if (isnan(v)) v = INFINITY;
        if (bi < 0 || v < bv) { bv = v; bi = i; }
    }
    sv[threadIdx.x] = bv;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const double ov = sv[threadIdx.x + w];
            const int64_t oi = si[threadIdx.x + w];
            const double mv = sv[threadIdx.x];
            const int64_t mi = si[threadIdx.x];
            const bool take = oi >= 0 && (mi < 0 || ov < mv || (ov == mv && oi < mi));
            if (take) { sv[threadIdx.x] = ov; si[threadIdx.x] = oi; }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        best->cost = sv[0];
        best->index = si[0] < 0 ? -1 : offset + si[0];
    }
}

// The selection exchange without a host round trip: every rank writes the winner's row if it owns
// it and zeros otherwise; a sum all-reduce then hands every rank the winner's row exactly (x + 0 = x).
__global__ void winner_row_kernel(const mpcd_best *best, int64_t lo, int64_t n_local, const float *rows, int row_len,
                                  float *out)
{
    const int64_t idx = best->index - lo;
    const bool own = idx >= 0 && idx < n_local;
    for (int i = threadIdx.x; i < row_len; i += blockDim.x) out[i] = own ? rows[idx * row_len + i] : 0.f;
}

}  // namespace

hipError_t launch_winner_row(const mpcd_best *best, int64_t lo, int64_t n_local, const float *rows, int row_len,
                             float *out, hipStream_t stream)
{
    hipLaunchKernelGGL(winner_row_kernel, dim3(1), dim3(256), 0, stream, best, lo, n_local, rows, row_len, out);
    return hipGetLastError();
}

hipError_t launch_clip_flag(const float *x, int64_t n, int *flag_dev, unsigned *ws, hipStream_t stream)
{
    const int64_t blocks = std::min<int64_t>(512, (n + 1023) / 1024);
    hipLaunchKernelGGL(clip_flag_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, stream, x, n, flag_dev,
                       ws);
    return hipGetLastError();
}

hipError_t launch_unnormalize(const float *x, int64_t n, int dim, const int *flag_dev, const float *mn_host,
                              const float *mx_host, float *out, hipStream_t stream)
{
    MinMax lim;
    for (int i = 0; i < 16; ++i) {
        lim.mn[i] = i < dim ? mn_host[i] : 0.f;
        lim.mx[i] = i < dim ? mx_host[i] : 0.f;
    }
    const int64_t blocks = std::min<int64_t>(4096, (n + 255) / 256);
    hipLaunchKernelGGL(unnormalize_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, stream, x, n,
                       dim, flag_dev, lim, out);
    return hipGetLastError();
}

hipError_t launch_rollout_cost(const mpcd_system_desc &d, const double *x0_host, const double *x0_dev, int64_t group,
                               const float *u_norm, const float *umin_host, const float *umax_host, const int *flag_dev,
                               int64_t batch, int H, double *cost, hipStream_t stream, const RolloutSelect *sel)
{
    if (group < 1) group = batch;
    SysK S = {};
    S.system = d.system;
    S.cost_kind = d.cost_kind;
    S.nx = d.n_x;
    S.nu = d.n_u;
    for (int i = 0; i < 24; ++i) S.params[i] = d.params[i];
    for (int i = 0; i < 12; ++i) { S.Q[i] = d.Q[i]; S.P[i] = d.P[i]; S.xr[i] = d.x_ref[i]; }
    for (int i = 0; i < 4; ++i) S.R[i] = d.R[i];
    for (int i = 0; i < d.n_x; ++i) S.x0[i] = x0_host ? x0_host[i] : 0.0;
    for (int i = 0; i < d.n_u; ++i) { S.umin[i] = umin_host[i]; S.umax[i] = umax_host[i]; }
    const size_t lds = sizeof(float) * RT_THREADS * (H * d.n_u + 1);
    SelectK K = {};
    if (sel) {
        if (group != batch || sel->n_part < (batch + RT_THREADS - 1) / RT_THREADS) return hipErrorInvalidValue;
        K = SelectK{sel->best,   sel->row_out, sel->part_cost, sel->part_idx, sel->counter,   sel->offset,
                    sel->code_out, sel->clip_src, sel->clip_n,   sel->host_out, sel->host_flag, sel->host_seq};
    }
    const dim3 grid((unsigned)((batch + RT_THREADS - 1) / RT_THREADS));
#define MPCD_ROLLOUT(SYS_)                                                                                          \
    case SYS_:                                                                                                      \
        if (d.n_x != SysDim<SYS_>::NX || d.n_u != SysDim<SYS_>::NU) return hipErrorInvalidValue;                    \
        if (sel)                                                                                                    \
            hipLaunchKernelGGL((rollout_cost_kernel<SYS_, true>), grid, dim3(RT_THREADS), lds, stream, S, u_norm,   \
                               flag_dev, x0_dev, group, batch, H, cost, K);                                         \
        else                                                                                                        \
            hipLaunchKernelGGL((rollout_cost_kernel<SYS_, false>), grid, dim3(RT_THREADS), lds, stream, S, u_norm,  \
                               flag_dev, x0_dev, group, batch, H, cost, K);                                         \
        break;
    switch (d.system) {
        MPCD_ROLLOUT(MPCD_SYS_CARTPOLE_LIN5)
        MPCD_ROLLOUT(MPCD_SYS_CARTPOLE_NL5)
        MPCD_ROLLOUT(MPCD_SYS_CARTPOLE_ZOH4)
        MPCD_ROLLOUT(MPCD_SYS_DOUBLE_INT2D)
        MPCD_ROLLOUT(MPCD_SYS_PENDULUM)
        MPCD_ROLLOUT(MPCD_SYS_QUADROTOR12)
    default: return hipErrorInvalidValue;
    }
#undef MPCD_ROLLOUT
    return hipGetLastError();
}

hipError_t launch_argmin(const double *cost, int64_t n, int64_t offset, mpcd_best *best, hipStream_t stream)
{
    hipLaunchKernelGGL(argmin_kernel, dim3(1), dim3(1024), 0, stream, cost, n, offset, best);
    return hipGetLastError();
}

hipError_t launch_clip_flags(const float *x, int64_t n_groups, int64_t group_elems, int *flags_dev, hipStream_t stream)
{
    if (n_groups > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(clip_flags_kernel, dim3((unsigned)n_groups), dim3(256), 0, stream, x, group_elems, flags_dev);
    return hipGetLastError();
}

hipError_t launch_normalize_states(const double *x, int64_t M, int C, const float *mn_host, const float *mx_host,
                                   float *out, hipStream_t stream)
{
    NormK nk;
    for (int i = 0; i < 16; ++i) {
        nk.mn[i] = i < C ? (double)mn_host[i] : 0.0;
        nk.den[i] = i < C ? (double)(mx_host[i] - mn_host[i]) : 1.0;  // fp32 subtraction, then promoted
    }
    const int64_t n = M * C;
    hipLaunchKernelGGL(normalize_states_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, M, C, nk, out);
    return hipGetLastError();
}

hipError_t launch_control_step(const mpcd_system_desc &d, double *x_dev, int64_t M, int64_t group, const float *u_norm,
                               int H, const double *cost, const float *umin_host, const float *umax_host,
                               const int *flags_dev, int select_first, int decimals, double *u_applied,
                               int64_t *best_idx, double *best_cost, hipStream_t stream)
{
    SysK S = {};
    S.system = d.system;
    S.cost_kind = d.cost_kind;
    S.nx = d.n_x;
    S.nu = d.n_u;
    for (int i = 0; i < 24; ++i) S.params[i] = d.params[i];
    for (int i = 0; i < d.n_u; ++i) {
        S.umin[i] = umin_host[i];
        S.umax[i] = umax_host[i];
    }
#define MPCD_CSTEP(SYS_)                                                                                         \
    case SYS_:                                                                                                   \
        if (d.n_x != SysDim<SYS_>::NX || d.n_u != SysDim<SYS_>::NU) return hipErrorInvalidValue;                 \
        hipLaunchKernelGGL(control_step_kernel<SYS_>, dim3((unsigned)M), dim3(CS_THREADS), 0, stream, S, x_dev, group, \
                           u_norm, H, cost, flags_dev, select_first, decimals, u_applied, best_idx, best_cost);  \
        break;
    switch (d.system) {
        MPCD_CSTEP(MPCD_SYS_CARTPOLE_LIN5)
        MPCD_CSTEP(MPCD_SYS_CARTPOLE_NL5)
        MPCD_CSTEP(MPCD_SYS_CARTPOLE_ZOH4)
        MPCD_CSTEP(MPCD_SYS_DOUBLE_INT2D)
        MPCD_CSTEP(MPCD_SYS_PENDULUM)
        MPCD_CSTEP(MPCD_SYS_QUADROTOR12)
    default: return hipErrorInvalidValue;
    }
#undef MPCD_CSTEP
    return hipGetLastError();
}
