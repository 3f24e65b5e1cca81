// Persistent CFG-DDPM / DDIM sampler for the MLP noise-net on gfx950.
//
// One launch runs every denoise step for every candidate. A 256-thread
// workgroup owns 32 "rows": for CFG (NB = 2) 16 candidates x {context, masked context}
// (the two forwards of p_mean_variance_CFG, diffusion_model_base.py:164-178, batched as rows),
// for the 3-arg net (NB = 1) 32 candidates. Activations never leave LDS; the trajectory x stays
// in LDS across all steps; weights stream from L2 into VGPRs one layer ahead of use.
//
// Net (build-defined CFG MLP, SURVEY §8a A11 = PointUnet temporal_unet.py:489-550 on [B, H*d]):
//   6 TemporalBlockMLP (layers.py:358-385): y = Mish(L2(Mish(L1 x)) + cond_mlp(c)); downs 3,
//   mid 1, ups 2 with cat(x, skip); final MLP(32, H*d, act=identity) = 2 Linear. 14 Linear total.
// cond_mlp(c) = Linear(Mish(cat(t_emb, ctx))) is split exactly into a per-step table (time part +
// bias, tproj) and a per-candidate table (context part, cproj) built by the prologue kernels.
//
// GEMM: D = W . act^T on v_mfma_f32_16x16x4_f32 (exact f32, fmaf-chain numerics): A = W rows (out
// features), B = activation rows. A lane's float4 of W and float4 of act cover 4 k each, so one
// 16-k block = 4 MFMAs; the k permutation is the same for A and B. Output lane layout: 4 consecutive
// features of one row -> one ds_write_b128.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "mlp_common.h"
#if !defined(MPCD_VARIANT) && (defined(MPCD_DIAG_NOMFMA) || defined(MPCD_DIAG_NOMISH))
#error "wrong-result timing diagnostics build only as an experiment variant (build.py variant: -DMPCD_VARIANT)"
#endif

namespace {
using namespace mlpc;

constexpr int ROWS = 32;
constexpr int THREADS = 256;
constexpr int CP_STRIDE = COND_TOTAL + 4;  // LDS cproj row stride (448 = 0 mod 64 banks: 16-way conflict)
enum { SPLIT = 0, PAIRED = 1 };

// ---- LDS layout (floats). Row strides are width + 4 so the 16 rows a ds_read_b128 lane group
// touches land on different 16-byte bank slots.
template <int D0, int NB>
struct Lds {
    static constexpr int CPW = ROWS / NB;          // candidates per workgroup
    static constexpr int SX = D0 + 4, ST1 = 132, SS1 = 68, SC1 = 132, SC0 = 260;  // all = 4 mod 64 (banks)
    static constexpr int XB = 0;
    static constexpr int T1 = XB + CPW * SX;
    static constexpr int S1 = T1 + ROWS * ST1;
    static constexpr int C1 = S1 + ROWS * SS1;
    static constexpr int C0 = C1 + ROWS * SC1;
    static constexpr int TP = C0 + ROWS * SC0;     // this step's tproj [448]
    static constexpr int BIC = TP + COND_TOTAL;    // biases of the cond layers in tproj column order
    static constexpr int BI = BIC + COND_TOTAL;    // all 14 biases
    static constexpr int AMX = BI + Arch<D0>::btotal();  // uint32 [ROWS]: chain |x| maxima
    static constexpr int CP = AMX + ROWS;          // per-candidate cproj [CPW][448]
    static constexpr int total(bool ctx) { return CP + (ctx ? CPW * CP_STRIDE : 0); }
};

template <int N>
constexpr int mode_for() { return N == 32 ? SPLIT : PAIRED; }

template <int K, int N, int MODE>
struct WFrag {
    static constexpr int NT = N / 16;
    static constexpr int T = MODE == SPLIT ? NT / 2 : (NT + 3) / 4;
    static constexpr int KB = K / 16;
    f32x4 v[T][KB];
};

template <int K, int N, int MODE>
MPCD_DEV int ntile_of(int wave, int j)
{
    return MODE == SPLIT ? (wave >> 1) + 2 * j : wave + 4 * j;
}

// Weight fragments stream in through buffer loads: ONE wave-uniform descriptor per layer (built
// from readfirstlane'd scalars, T20), the per-lane part is lane*16 in a single VGPR and each
// (n-tile, k-block) chunk offset is a scalar soffset. A flat/global form kept one 64-bit VGPR
// address per chunk live across the step loop (hundreds of VGPRs, spills to scratch).
template <int K, int N, int MODE>
MPCD_DEV void load_w(WFrag<K, N, MODE> &f, const float *__restrict__ wp, int wave, int lane16)
{
    constexpr int KB = K / 16, NT = N / 16;
    const uint64_t a = (uint64_t)wp;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(((uint64_t)hi << 32) | lo), (short)0, (int)(K * N * sizeof(float)), 0x00020000);
#pragma unroll
    for (int j = 0; j < WFrag<K, N, MODE>::T; ++j) {
        const int nt = ntile_of<K, N, MODE>(wave, j);
        if (MODE == PAIRED && NT % 4 != 0 && nt >= NT) continue;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            const int soff = __builtin_amdgcn_readfirstlane((nt * KB + kb) * 1024);
            const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, lane16, soff, 0);
            f.v[j][kb] = __builtin_bit_cast(f32x4, r);
        }
    }
}

// Two independent 16-k chains, issued alternately: a v_mfma_f32_16x16x4_f32 whose C operand is the
// previous MFMA's result waits 40 cycles instead of issuing at the 32-cycle pipe rate.
MPCD_DEV void mfma4x2(const f32x4 &wa, const f32x4 &aa, f32x4 &acca, const f32x4 &wb, const f32x4 &ab, f32x4 &accb)
{
    acca = __builtin_amdgcn_mfma_f32_16x16x4f32(wa.x, aa.x, acca, 0, 0, 0);
    accb = __builtin_amdgcn_mfma_f32_16x16x4f32(wb.x, ab.x, accb, 0, 0, 0);
    acca = __builtin_amdgcn_mfma_f32_16x16x4f32(wa.y, aa.y, acca, 0, 0, 0);
    accb = __builtin_amdgcn_mfma_f32_16x16x4f32(wb.y, ab.y, accb, 0, 0, 0);
    acca = __builtin_amdgcn_mfma_f32_16x16x4f32(wa.z, aa.z, acca, 0, 0, 0);
    accb = __builtin_amdgcn_mfma_f32_16x16x4f32(wb.z, ab.z, accb, 0, 0, 0);
    acca = __builtin_amdgcn_mfma_f32_16x16x4f32(wa.w, aa.w, acca, 0, 0, 0);
    accb = __builtin_amdgcn_mfma_f32_16x16x4f32(wb.w, ab.w, accb, 0, 0, 0);
}

MPCD_DEV f32x4 mfma4(const f32x4 &w, const f32x4 &a, f32x4 acc)
{
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, a.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, a.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, a.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, a.w, acc, 0, 0, 0);
    return acc;
}

// Hidden layer. SPLIT (N = 32): wave w -> column tile (w & 1), n-tiles (w >> 1) + 2j.
// PAIRED (N >= 64): wave w -> n-tiles w + 4j for BOTH column tiles, so each weight register feeds
// two MFMAs and a wave holds only a quarter of the layer's weights.
// in_shared: both column tiles read rows 0..15 (layer 0 with CFG: both branches see the same x).
//
// The accumulators start from `init` (LDS, per output feature): the layer bias, or for the cond
// layers tproj + bias (the time part of cond_mlp and the Linear bias, pre-summed when the step's
// tproj is staged), so the epilogue adds only the context part on the context rows. Every wave
// issues two independent accumulation chains alternately (two column tiles of one n-tile when
// T = 2, else the even / odd k-blocks of one tile, summed at the end): f32 MFMA and VALU share the
// SIMD's issue on gfx950, so VALU ops per output element are what the epilogue minimises.
template <int K, int N, int MODE, int EPI, int NB>
MPCD_DEV void hidden_layer(const WFrag<K, N, MODE> &f, const float *init, const float *in, int in_stride,
                           bool in_shared, float *out, int out_stride, const float *cp, int cond_j, bool has_ctx,
                           int wave, int lane)
{
    constexpr int T = WFrag<K, N, MODE>::T, KB = K / 16, NT = N / 16;
    constexpr int NCT = MODE == SPLIT ? 1 : 2;
    static_assert(MODE == SPLIT || NT % 4 == 0, "PAIRED hidden layers need N % 64 == 0");
    static_assert(KB % 2 == 0, "even / odd k-block chains need K % 32 == 0");
    static_assert(T <= 2 && (T == 1 || NCT == 2), "group layout");
    constexpr bool BYJ = T == 2;        // group = n-tile j, chains = the two column tiles
    constexpr int G = BYJ ? T : NCT;    // else group = column tile, chains = even / odd k-blocks
    const int col = lane & 15, q = lane >> 4;

    f32x4 a[NCT][KB];
#pragma unroll
    for (int c = 0; c < NCT; ++c) {
        const int ct = MODE == SPLIT ? (wave & 1) : c;
        const float *arow = in + (size_t)((in_shared ? 0 : ct * 16) + col) * in_stride + 4 * q;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) a[c][kb] = *reinterpret_cast<const f32x4 *>(arow + kb * 16);
    }
    f32x4 i4[T];
#pragma unroll
    for (int j = 0; j < T; ++j) i4[j] = *reinterpret_cast<const f32x4 *>(init + ntile_of<K, N, MODE>(wave, j) * 16 + 4 * q);

    f32x4 acc[G][2];
#ifdef MPCD_DIAG_NOMFMA
    // timing diagnostic only (wrong results): no MFMAs, activations folded in so loads stay live
#pragma unroll
    for (int g = 0; g < G; ++g) {
        acc[g][0] = i4[BYJ ? g : 0] + a[BYJ ? 0 : g][0];
        acc[g][1] = a[BYJ ? 1 % NCT : g][KB - 1] + f.v[BYJ ? g : 0][KB - 1];
    }
    if (false)
#endif
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if (BYJ) {
            acc[g][0] = acc[g][1] = i4[g];
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) mfma4x2(f.v[g][kb], a[0][kb], acc[g][0], f.v[g][kb], a[1][kb], acc[g][1]);
        } else {
            acc[g][0] = i4[0];
            acc[g][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kb = 0; kb < KB; kb += 2)
                mfma4x2(f.v[0][kb], a[g][kb], acc[g][0], f.v[0][kb + 1], a[g][kb + 1], acc[g][1]);
        }
    }
#pragma unroll
    for (int t = 0; t < T * NCT; ++t) {
        const int j = t / NCT, c = t % NCT;
        const int ct = MODE == SPLIT ? (wave & 1) : c;
        const int n = ntile_of<K, N, MODE>(wave, j) * 16 + 4 * q;
        f32x4 v = BYJ ? acc[j][c] : acc[c][0] + acc[c][1];
        // context part of cond_mlp: NB == 2 only on the context branch (column tile 0; the masked
        // tile takes the time part alone, already in the accumulator), NB == 1 on every row. SPLIT
        // layers know their tile at run time: multiply-add by an exact 0/1 factor, no branch.
        if (EPI == EPI_CMISH && has_ctx && (NB == 1 || MODE == SPLIT || c == 0)) {
            const int cand = NB == 2 ? col : ct * 16 + col;
            const f32x4 cpv = *reinterpret_cast<const f32x4 *>(cp + cand * CP_STRIDE + cond_off(cond_j) + n);
            if (NB == 2 && MODE == SPLIT) {
                const float on = ct == 0 ? 1.0f : 0.0f;
                v.x = __builtin_fmaf(cpv.x, on, v.x);
                v.y = __builtin_fmaf(cpv.y, on, v.y);
                v.z = __builtin_fmaf(cpv.z, on, v.z);
                v.w = __builtin_fmaf(cpv.w, on, v.w);
            } else {
                v = v + cpv;
            }
        }
#ifndef MPCD_DIAG_NOMISH
        if (EPI != EPI_NONE) {
            v.x = mish_scalar(v.x);
            v.y = mish_scalar(v.y);
            v.z = mish_scalar(v.z);
            v.w = mish_scalar(v.w);
        }
#endif
        *reinterpret_cast<f32x4 *>(out + (size_t)(ct * 16 + col) * out_stride + n) = v;
    }
}

template <int D0, int SMODE, bool CTX>
struct MlpKernel {
    static constexpr int NB = (SMODE == MODE_DDIM || SMODE == MODE_EPS1) ? 1 : 2;
    static constexpr bool IS_DDPM = SMODE == MODE_DDPM_CFG || SMODE == MODE_DDPM_XN;
    using A = Arch<D0>;
    using L = Lds<D0, NB>;
    static constexpr int CPW = L::CPW;
    static constexpr int QUADS = D0 / 4;  // float4 quads per candidate trajectory

    // final Linear (32 -> D0) in PAIRED mode + the denoise update, x kept in LDS
    static MPCD_DEV void final_and_update(const WFrag<32, D0, PAIRED> &f, const float *__restrict__ bias, float *lds,
                                          const MlpSampleArgs &p, const StepPlan &sp, int s, int64_t cand0,
                                          const f32x4 (&nz)[WFrag<32, D0, PAIRED>::T][NB], uint32_t (&am)[2],
                                          int wave, int lane)
    {
        constexpr int T = WFrag<32, D0, PAIRED>::T, NT = D0 / 16;
        const int col = lane & 15, q = lane >> 4;
        f32x4 acc[T][2];
#pragma unroll
        for (int j = 0; j < T; ++j) {  // accumulators start from the bias (idle tiles read n-tile 0, unused)
            const int nt = (NT % 4 == 0 || wave + 4 * j < NT) ? wave + 4 * j : 0;
            acc[j][0] = acc[j][1] = *reinterpret_cast<const f32x4 *>(bias + nt * 16 + 4 * q);
        }
        const float *arow0 = lds + L::T1 + (size_t)col * L::ST1 + 4 * q;
        const float *arow1 = arow0 + 16 * L::ST1;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            const f32x4 a0 = *reinterpret_cast<const f32x4 *>(arow0 + kb * 16);
            const f32x4 a1 = *reinterpret_cast<const f32x4 *>(arow1 + kb * 16);
#pragma unroll
            for (int j = 0; j < T; ++j)
                if (NT % 4 == 0 || wave + 4 * j < NT) mfma4x2(f.v[j][kb], a0, acc[j][0], f.v[j][kb], a1, acc[j][1]);
        }
        const bool last = s == p.n_steps - 1;
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const int nt = wave + 4 * j;
            if (NT % 4 != 0 && nt >= NT) continue;
            const int n = nt * 16 + 4 * q;
#pragma unroll
            for (int g = 0; g < (NB == 2 ? 1 : 2); ++g) {
                // NB == 2: one candidate per lane column, eps_c = tile 0, eps_u = tile 1
                // NB == 1: column tile g holds candidates 16g..16g+15
                const int cl = NB == 2 ? col : g * 16 + col;
                float *xp = lds + L::XB + (size_t)cl * L::SX + n;
                const f32x4 x = *reinterpret_cast<const f32x4 *>(xp);
                const f32x4 ec = acc[j][NB == 2 ? 0 : g];
                const f32x4 eu = acc[j][1];
                if (SMODE == MODE_EPS || SMODE == MODE_EPS1) {
                    const int64_t gc = cand0 + cl;
                    if (gc < p.batch) {
                        *reinterpret_cast<f32x4 *>(p.x_out + (size_t)gc * D0 + n) = ec;
                        if (SMODE == MODE_EPS) *reinterpret_cast<f32x4 *>(p.chain + (size_t)gc * D0 + n) = eu;
                    }
                    continue;
                }
                f32x4 xn;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float xv = x[r];
                    float o;
                    if (IS_DDPM) {
                        const float x0c = sp.a * xv - sp.b * ec[r];
                        const float x0u = sp.a * xv - sp.b * eu[r];
                        float x0 = p.wp1 * x0c - p.wf * x0u;
                        x0 = clamp1(x0);
                        const float mean = sp.c1 * x0 + sp.c2 * xv;
                        o = (sp.flags & PLAN_NOISE) ? mean + sp.std * nz[j][0][r] : mean;
                    } else if (SMODE == MODE_DDIM_CFG) {
                        float x0 = p.wp1 * (sp.a * xv - sp.b * ec[r]) - p.wf * (sp.a * xv - sp.b * eu[r]);
                        if (p.clamp_x0) x0 = clamp1(x0);
                        const float e = p.wp1 * ec[r] - p.wf * eu[r];
                        o = (sp.flags & PLAN_FINAL) ? x0 : x0 * sp.sqan + sp.cn * e;
                    } else {  // MODE_DDIM, 3-arg net
                        float x0 = sp.a * xv - sp.b * ec[r];
                        if (p.clamp_x0) x0 = clamp1(x0);
                        o = (sp.flags & PLAN_FINAL) ? x0 : x0 * sp.sqan + sp.cn * ec[r];
                    }
                    xn[r] = o;
                    am[g] = max(am[g], max(abs_bits(xv), abs_bits(o)));  // chain |x| max (x_T .. x_0)
                }
                *reinterpret_cast<f32x4 *>(xp) = xn;
                const int64_t gc = cand0 + cl;
                if (gc < p.batch) {
                    if (p.chain)
                        *reinterpret_cast<f32x4 *>(p.chain + ((size_t)(s + 1) * p.batch + gc) * D0 + n) = xn;
                    if (last) *reinterpret_cast<f32x4 *>(p.x_out + (size_t)gc * D0 + n) = xn;
                }
            }
        }
    }

    // noise of step s (slice s+1) for this lane's quads, fetched one step ahead of use
    static MPCD_DEV void fetch_noise(f32x4 (&nz)[WFrag<32, D0, PAIRED>::T][NB], const MlpSampleArgs &p,
                                     const StepPlan &sp, int s, int64_t cand0, int wave, int lane)
    {
        constexpr int T = WFrag<32, D0, PAIRED>::T, NT = D0 / 16;
#pragma unroll
        for (int j = 0; j < T; ++j)
#pragma unroll
            for (int g = 0; g < NB; ++g) nz[j][g] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (!IS_DDPM || !(sp.flags & PLAN_NOISE)) return;  // DDIM: sigma = 0
        const int col = lane & 15, q = lane >> 4;
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const int nt = wave + 4 * j;
            if (NT % 4 != 0 && nt >= NT) continue;
            const int n = nt * 16 + 4 * q;
            const int64_t gc = cand0 + col;  // DDPM-CFG only: NB == 2, one candidate per column
            if (gc >= p.batch) continue;
            if (SMODE == MODE_DDPM_XN)
                nz[j][0] = *reinterpret_cast<const f32x4 *>(p.noise + ((size_t)(s + 1) * p.batch + gc) * D0 + n);
            else
                nz[j][0] = philox_normal4(p.seed, (uint64_t)(p.global_offset + gc), (uint32_t)(s + 1), (uint32_t)(n >> 2));
        }
    }

    static MPCD_DEV void dump(const MlpSampleArgs &p, const float *buf, int stride, int width, int layer)
    {
        if (SMODE != MODE_EPS || !p.dbg || blockIdx.x != 0) return;
        lds_barrier();
        for (int i = threadIdx.x; i < ROWS * width; i += THREADS) {
            const int r = i / width, c = i - r * width;
            p.dbg[(size_t)layer * ROWS * 256 + r * 256 + c] = buf[r * stride + c];
        }
    }

    static MPCD_DEV void run(const MlpSampleArgs &p)
    {
        extern __shared__ float lds[];
        const int lane = threadIdx.x & 63;
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const int64_t cand0 = (int64_t)blockIdx.x * CPW;
        constexpr bool has_ctx = CTX;
        int lane16 = lane * 16;
        const float *wp = p.wpack;
        int wofs = 0;
        auto W = [&](int l) { return wp + wofs + A::woff(l); };
        auto Bs = [&](int l) { return lds + L::BI + A::boff(l); };

        // biases of every layer -> LDS (read in each epilogue instead of a global round trip)
        for (int l = 0; l < NLAYER; ++l)
            for (int i = threadIdx.x; i < A::N[l]; i += THREADS) lds[L::BI + A::boff(l) + i] = wp[A::woff(l) + A::K[l] * A::N[l] + i];
        // biases of the cond layers (1, 3, ..., 11) laid out like tproj: TP = tproj[s] + BIC per step
        for (int j = 0; j < 6; ++j)
            for (int i = threadIdx.x; i < A::N[2 * j + 1]; i += THREADS)
                lds[L::BIC + cond_off(j) + i] = wp[A::woff(2 * j + 1) + A::K[2 * j + 1] * A::N[2 * j + 1] + i];
        // per-candidate context projections (constant over the denoise loop)
        if (has_ctx) {
            for (int i = threadIdx.x; i < CPW * COND_TOTAL; i += THREADS) {
                const int c = i / COND_TOTAL, k = i - c * COND_TOTAL;
                const int64_t gc = cand0 + c;
                lds[L::CP + c * CP_STRIDE + k] = gc < p.batch ? p.cproj[(size_t)(p.cproj_stride ? gc : 0) * COND_TOTAL + k] : 0.f;
            }
        }
        if (threadIdx.x < CPW) reinterpret_cast<uint32_t *>(lds + L::AMX)[threadIdx.x] = 0u;
        uint32_t am[2] = {0u, 0u};
        // x_T
        for (int i = threadIdx.x; i < CPW * QUADS; i += THREADS) {
            const int c = i / QUADS, qd = i - c * QUADS;
            const int64_t gc = cand0 + c;
            f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
            if (gc < p.batch) {
                z = p.noise ? *reinterpret_cast<const f32x4 *>(p.noise + (size_t)gc * D0 + qd * 4)
                            : philox_normal4(p.seed, (uint64_t)(p.global_offset + gc), 0u, (uint32_t)qd);
                if (p.chain && SMODE != MODE_EPS) *reinterpret_cast<f32x4 *>(p.chain + (size_t)gc * D0 + qd * 4) = z;
            }
            *reinterpret_cast<f32x4 *>(lds + L::XB + c * L::SX + qd * 4) = z;
        }

        WFrag<A::K[0], A::N[0], mode_for<A::N[0]>()> w0;
        load_w(w0, W(0), wave, lane16);
        constexpr int NZT = WFrag<32, D0, PAIRED>::T;
        f32x4 nz[NZT][NB];
        StepPlan sp = load_plan(p.plan, 0);
        fetch_noise(nz, p, sp, 0, cand0, wave, lane);
        // tproj of step s, prefetched one step ahead (threads >= COND_TOTAL/4 load a duplicate, unused)
        const int tpi = threadIdx.x < COND_TOTAL / 4 ? (int)threadIdx.x : 0;
        f32x4 tpre = reinterpret_cast<const f32x4 *>(p.tproj)[tpi];

#ifdef MPCD_PROF_LAYERS
        // experiment build only: per-wave shader-clock cycles of each layer (work, then barrier wait)
        uint64_t tacc[2 * 16] = {};
        const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
        uint64_t tprev = __builtin_readcyclecounter();
        const uint64_t ct0 = tprev;
        auto bar = [&](int k) {
            uint64_t t = __builtin_readcyclecounter();
            tacc[2 * k] += t - tprev;
            lds_barrier();
            tprev = __builtin_readcyclecounter();
            tacc[2 * k + 1] += tprev - t;
        };
#else
        auto bar = [](int) { lds_barrier(); };
#endif
        for (int s = 0; s < p.n_steps; ++s) {
            // Launder the weight base every step: the weights are loop-invariant, and without this
            // LICM hoists all 14 layers' loads out of the step loop (hundreds of live VGPRs -> spills).
            asm volatile("" : "+s"(wofs), "+v"(lane16));
            WFrag<A::K[1], A::N[1], mode_for<A::N[1]>()> w1;
            load_w(w1, W(1), wave, lane16);
            bar(0);
            // this step's time projections + cond-layer biases -> LDS (first read by layer 1, after
            // the next barrier); fetch the next step's
            static_assert(COND_TOTAL / 4 <= THREADS, "tproj staging");
            if (threadIdx.x < COND_TOTAL / 4)
                reinterpret_cast<f32x4 *>(lds + L::TP)[tpi] = tpre + reinterpret_cast<const f32x4 *>(lds + L::BIC)[tpi];
            tpre = reinterpret_cast<const f32x4 *>(p.tproj + (size_t)(s + 1 < p.n_steps ? s + 1 : s) * COND_TOTAL)[tpi];
            const float *tp = lds + L::TP, *cp = lds + L::CP;
            hidden_layer<A::K[0], A::N[0], mode_for<A::N[0]>(), EPI_MISH, NB>(w0, Bs(0), lds + L::XB, L::SX, NB == 2, lds + L::T1, L::ST1, cp, 0, has_ctx, wave, lane);
            dump(p, lds + L::T1, L::ST1, 32, 0);
            WFrag<A::K[2], A::N[2], mode_for<A::N[2]>()> w2;
            load_w(w2, W(2), wave, lane16);
            bar(1);
            hidden_layer<A::K[1], A::N[1], mode_for<A::N[1]>(), EPI_CMISH, NB>(w1, tp + cond_off(0), lds + L::T1, L::ST1, false, lds + L::S1, L::SS1, cp, 0, has_ctx, wave, lane);
            dump(p, lds + L::S1, L::SS1, 32, 1);
            WFrag<A::K[3], A::N[3], mode_for<A::N[3]>()> w3;
            load_w(w3, W(3), wave, lane16);
            bar(2);
            hidden_layer<A::K[2], A::N[2], mode_for<A::N[2]>(), EPI_MISH, NB>(w2, Bs(2), lds + L::S1, L::SS1, false, lds + L::T1, L::ST1, cp, 0, has_ctx, wave, lane);
            dump(p, lds + L::T1, L::ST1, 64, 2);
            WFrag<A::K[4], A::N[4], mode_for<A::N[4]>()> w4;
            load_w(w4, W(4), wave, lane16);
            bar(3);
            hidden_layer<A::K[3], A::N[3], mode_for<A::N[3]>(), EPI_CMISH, NB>(w3, tp + cond_off(1), lds + L::T1, L::ST1, false, lds + L::C1 + 64, L::SC1, cp, 1, has_ctx, wave, lane);
            dump(p, lds + L::C1 + 64, L::SC1, 64, 3);
            WFrag<A::K[5], A::N[5], mode_for<A::N[5]>()> w5;
            load_w(w5, W(5), wave, lane16);
            bar(4);
            hidden_layer<A::K[4], A::N[4], mode_for<A::N[4]>(), EPI_MISH, NB>(w4, Bs(4), lds + L::C1 + 64, L::SC1, false, lds + L::T1, L::ST1, cp, 0, has_ctx, wave, lane);
            dump(p, lds + L::T1, L::ST1, 128, 4);
            WFrag<A::K[6], A::N[6], mode_for<A::N[6]>()> w6;
            load_w(w6, W(6), wave, lane16);
            bar(5);
            hidden_layer<A::K[5], A::N[5], mode_for<A::N[5]>(), EPI_CMISH, NB>(w5, tp + cond_off(2), lds + L::T1, L::ST1, false, lds + L::C0 + 128, L::SC0, cp, 2, has_ctx, wave, lane);
            dump(p, lds + L::C0 + 128, L::SC0, 128, 5);
            WFrag<A::K[7], A::N[7], mode_for<A::N[7]>()> w7;
            load_w(w7, W(7), wave, lane16);
            bar(6);
            hidden_layer<A::K[6], A::N[6], mode_for<A::N[6]>(), EPI_MISH, NB>(w6, Bs(6), lds + L::C0 + 128, L::SC0, false, lds + L::T1, L::ST1, cp, 0, has_ctx, wave, lane);
            dump(p, lds + L::T1, L::ST1, 128, 6);
            WFrag<A::K[8], A::N[8], mode_for<A::N[8]>()> w8;
            load_w(w8, W(8), wave, lane16);
            bar(7);
            hidden_layer<A::K[7], A::N[7], mode_for<A::N[7]>(), EPI_CMISH, NB>(w7, tp + cond_off(3), lds + L::T1, L::ST1, false, lds + L::C0, L::SC0, cp, 3, has_ctx, wave, lane);
            dump(p, lds + L::C0, L::SC0, 128, 7);
            WFrag<A::K[9], A::N[9], mode_for<A::N[9]>()> w9;
            load_w(w9, W(9), wave, lane16);
            bar(8);
            hidden_layer<A::K[8], A::N[8], mode_for<A::N[8]>(), EPI_MISH, NB>(w8, Bs(8), lds + L::C0, L::SC0, false, lds + L::T1, L::ST1, cp, 0, has_ctx, wave, lane);
            dump(p, lds + L::T1, L::ST1, 64, 8);
            WFrag<A::K[10], A::N[10], mode_for<A::N[10]>()> w10;
            load_w(w10, W(10), wave, lane16);
            bar(9);
            hidden_layer<A::K[9], A::N[9], mode_for<A::N[9]>(), EPI_CMISH, NB>(w9, tp + cond_off(4), lds + L::T1, L::ST1, false, lds + L::C1, L::SC1, cp, 4, has_ctx, wave, lane);
            dump(p, lds + L::C1, L::SC1, 64, 9);
            WFrag<A::K[11], A::N[11], mode_for<A::N[11]>()> w11;
            load_w(w11, W(11), wave, lane16);
            bar(10);
            hidden_layer<A::K[10], A::N[10], mode_for<A::N[10]>(), EPI_MISH, NB>(w10, Bs(10), lds + L::C1, L::SC1, false, lds + L::T1, L::ST1, cp, 0, has_ctx, wave, lane);
            dump(p, lds + L::T1, L::ST1, 32, 10);
            WFrag<A::K[12], A::N[12], mode_for<A::N[12]>()> w12;
            load_w(w12, W(12), wave, lane16);
            bar(11);
            hidden_layer<A::K[11], A::N[11], mode_for<A::N[11]>(), EPI_CMISH, NB>(w11, tp + cond_off(5), lds + L::T1, L::ST1, false, lds + L::S1, L::SS1, cp, 5, has_ctx, wave, lane);
            dump(p, lds + L::S1, L::SS1, 32, 11);
            WFrag<A::K[13], A::N[13], PAIRED> w13;
            load_w(w13, W(13), wave, lane16);
            bar(12);
            hidden_layer<A::K[12], A::N[12], mode_for<A::N[12]>(), EPI_NONE, NB>(w12, Bs(12), lds + L::S1, L::SS1, false, lds + L::T1, L::ST1, cp, 0, has_ctx, wave, lane);
            dump(p, lds + L::T1, L::ST1, 32, 12);
            const StepPlan cur = sp;
            f32x4 nzc[NZT][NB];
#pragma unroll
            for (int j = 0; j < NZT; ++j)
#pragma unroll
                for (int g = 0; g < NB; ++g) nzc[j][g] = nz[j][g];
            if (s + 1 < p.n_steps) {
                sp = load_plan(p.plan, s + 1);
                fetch_noise(nz, p, sp, s + 1, cand0, wave, lane);
            }
            // next step's layer-0 weights; unconditional: a path-dependent load count makes the
            // compiler drain vmcnt(0) at the next use
            load_w(w0, W(0), wave, lane16);
            bar(13);
            final_and_update(w13, Bs(13), lds, p, cur, s, cand0, nzc, am, wave, lane);
        }
        if (SMODE != MODE_EPS && SMODE != MODE_EPS1 && p.chain_absmax) {
            const int col = lane & 15;
            store_chain_absmax<CPW, THREADS>(reinterpret_cast<uint32_t *>(lds + L::AMX), am, col, NB == 2 ? -1 : 16 + col,
                                             true, p.chain_absmax, cand0, p.batch);
        }
#ifdef MPCD_PROF_LAYERS
        {
            const uint64_t t = __builtin_readcyclecounter();
            tacc[2 * 15] += t - tprev;
            if (p.dbg && blockIdx.x < 8 && lane == 0)
                for (int i = 0; i < 32; ++i) p.dbg[(blockIdx.x * 4 + wave) * 32 + i] = (float)tacc[i];
            if (p.dbg && threadIdx.x == 0) {  // per-block loop start / end (memrealtime, low 32 bits)
                p.dbg[4096 + blockIdx.x * 2] = __builtin_bit_cast(float, (uint32_t)rt0);
                p.dbg[4096 + blockIdx.x * 2 + 1] = __builtin_bit_cast(float, (uint32_t)__builtin_amdgcn_s_memrealtime());
            }
            if (p.dbg && blockIdx.x < 8 && threadIdx.x == 0) {  // shader clock = d(memtime) / d(memrealtime) x 100 MHz
                p.dbg[8 * 4 * 32 + blockIdx.x * 2] = (float)(t - ct0);
                p.dbg[8 * 4 * 32 + blockIdx.x * 2 + 1] = (float)(__builtin_amdgcn_s_memrealtime() - rt0);
            }
        }
#endif
    }
};

template <int D0, int SMODE, bool CTX>
__global__ __launch_bounds__(THREADS, 1) void mlp_sample_kernel(const MlpSampleArgs p)
{
    MlpKernel<D0, SMODE, CTX>::run(p);
}

template <int D0, int SMODE, bool CTX>
hipError_t launch_impl(const MlpSampleArgs &a, hipStream_t stream)
{
    using L = Lds<D0, MlpKernel<D0, SMODE, CTX>::NB>;
    static_assert(sizeof(float) * L::total(CTX) <= 160 * 1024, "LDS budget (160 KiB per CU)");
    const size_t lds_bytes = sizeof(float) * L::total(CTX);
    if (hipError_t e = allow_max_lds<&mlp_sample_kernel<D0, SMODE, CTX>>(); e != hipSuccess) return e;
    const int64_t blocks = (a.batch + L::CPW - 1) / L::CPW;
    return launch_sampler_kernel(mlp_sample_kernel<D0, SMODE, CTX>, dim3((unsigned)blocks), dim3(THREADS), lds_bytes, stream, a);
}

template <int D0>
hipError_t launch_d0(const MlpSampleArgs &a, hipStream_t stream)
{
    const bool ctx = a.cproj != nullptr;
    switch (a.mode) {
    case MODE_DDPM_CFG:
        if (a.noise) return ctx ? launch_impl<D0, MODE_DDPM_XN, true>(a, stream) : launch_impl<D0, MODE_DDPM_XN, false>(a, stream);
        return ctx ? launch_impl<D0, MODE_DDPM_CFG, true>(a, stream) : launch_impl<D0, MODE_DDPM_CFG, false>(a, stream);
    case MODE_DDIM_CFG: return ctx ? launch_impl<D0, MODE_DDIM_CFG, true>(a, stream) : launch_impl<D0, MODE_DDIM_CFG, false>(a, stream);
    case MODE_DDIM: return ctx ? launch_impl<D0, MODE_DDIM, true>(a, stream) : launch_impl<D0, MODE_DDIM, false>(a, stream);
    case MODE_EPS: return ctx ? launch_impl<D0, MODE_EPS, true>(a, stream) : launch_impl<D0, MODE_EPS, false>(a, stream);
    case MODE_EPS1: return ctx ? launch_impl<D0, MODE_EPS1, true>(a, stream) : launch_impl<D0, MODE_EPS1, false>(a, stream);
    }
    return hipErrorInvalidValue;
}

}  // namespace

int mlp_packed_floats(int d0)
{
    switch (d0) {
    case 32: return Arch<32>::total();
    case 64: return Arch<64>::total();
    case 128: return Arch<128>::total();
    default: return -1;
    }
}

// Pack Linear l (torch weight [N][K], bias [N]) to the MFMA A-operand order:
// packed[((nt*KB + kb)*64 + lane)*4 + s] = W[nt*16 + (lane&15)][kb*16 + 4*(lane>>4) + s], then bias.
void mlp_pack_weights(int d0, const float *const *lin_w, const float *const *lin_b, float *out)
{
    const int Ks[NLAYER] = {d0, 32, 32, 64, 64, 128, 128, 128, 256, 64, 128, 32, 32, 32};
    const int Ns[NLAYER] = {32, 32, 64, 64, 128, 128, 128, 128, 64, 64, 32, 32, 32, d0};
    size_t o = 0;
    for (int l = 0; l < NLAYER; ++l) {
        const int K = Ks[l], N = Ns[l], KB = K / 16, NT = N / 16;
        for (int nt = 0; nt < NT; ++nt)
            for (int kb = 0; kb < KB; ++kb)
                for (int lane = 0; lane < 64; ++lane)
                    for (int s = 0; s < 4; ++s)
                        out[o + (((size_t)nt * KB + kb) * 64 + lane) * 4 + s] =
                            lin_w[l][(size_t)(nt * 16 + (lane & 15)) * K + kb * 16 + 4 * (lane >> 4) + s];
        o += (size_t)K * N;
        for (int n = 0; n < N; ++n) out[o + n] = lin_b[l][n];
        o += N;
    }
}

hipError_t launch_mlp_sampler(int d0, int nb, const MlpSampleArgs &a, hipStream_t stream)
{
    if ((nb == 1) != (a.mode == MODE_DDIM || a.mode == MODE_EPS1)) return hipErrorInvalidValue;
    switch (d0) {
    case 32: return launch_d0<32>(a, stream);
    case 64: return launch_d0<64>(a, stream);
    case 128: return launch_d0<128>(a, stream);
    }
    return hipErrorInvalidValue;
}
