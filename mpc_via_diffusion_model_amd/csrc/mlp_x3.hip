// Persistent CFG-DDPM / DDIM sampler for the MLP noise-net, fp32-accurate split-bf16 GEMMs.
//
// Same schedule as mlp_sampler.hip (one launch = every denoise step for every candidate; a
// 256-thread workgroup owns 32 rows = 16 candidates x {context, masked} for CFG or 32 candidates
// for the 3-arg net; activations and x stay in LDS; weights stream from L2 one layer ahead), but the
// 14 Linear layers run on v_mfma_f32_16x16x32_bf16 instead of the f32 MFMA.
//
// Why: on gfx950 the f32 MFMA runs at the f32 VALU rate and occupies the SIMD's vector issue for
// its whole 32 cycles, so the exact-f32 kernel is bound by MFMA + VALU issue.
// bf16 MFMA is 16x faster per MAC. Numerics stay fp32: every fp32 operand is split into three bf16
// terms, x = x0 + x1 + x2 (each level round-to-nearest on the remainder of the previous one, so the
// three carry x's 24-bit significand to ~2^-27), and every dot product accumulates the six partial
// products whose weight is at least 2^-16 of the leading one (x2w0, x1w1, x0w2, x1w0, x0w1, x0w0)
// in the fp32 accumulator. The dropped terms are <= 3 * 2^-24 relative; measured GEMM error
// (tests/test_gpu_mlp.py) is at or below the exact-f32 MFMA's. Weights are split once at load
// (host, exact); activations are split in each layer's epilogue (v_cvt_pk_bf16_f32 + subtractions)
// and stored in LDS as three bf16 planes.
//
// Net and conditioning as in mlp_sampler.hip. This variant takes a context shared by all candidates
// (mpc_step's case: one measured state per control step) or none; the time part, the Linear bias
// and the shared context part of every cond_mlp are pre-summed into the accumulator init per step
// (TPC: context rows, TPU: masked rows). Per-candidate contexts use the exact-f32 kernel.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>

#include "mlp_x3.h"

namespace {
using namespace mlpx3;

template <int D0, int SMODE, bool CTX, int R, int W = WAVES>
struct MlpX3 {
    static constexpr int NTHR = 64 * W;  // threads per workgroup
    static constexpr int NB = (SMODE == MODE_DDIM || SMODE == MODE_EPS1) ? 1 : 2;
    static constexpr bool IS_DDPM = SMODE == MODE_DDPM_CFG || SMODE == MODE_DDPM_XN;
    static_assert(R == 32 || R == 16, "32 or 16 rows per workgroup");
    static_assert(W == 8 || W == 4, "4 or 8 waves per workgroup");
    static constexpr bool H8 = W == 8 || R == 16;  // hidden8() for every layer (else the 4-wave hidden())
    using A = Arch<D0>;
    using L = Lds3<D0, NB, R>;
    // R = 16 with CFG: columns 0-7 are the context rows of candidates 0-7, 8-15 their masked rows
    static MPCD_DEV int cand_of(int ct, int col) { return NB == 2 ? (R == 16 ? (col & 7) : col) : ct * 16 + col; }
    static MPCD_DEV bool masked_of(int ct, int col) { return NB == 2 && (R == 16 ? col >= 8 : ct == 1); }
    static constexpr int CPW = L::CPW;
    static constexpr int QUADS = D0 / 4;
    using FW = WFrag3<32, D0, PAIRED>;
    using FWL = WLoad<32, D0, PAIRED>;
    static constexpr int NZT = FW::T;

    // Hidden layer l. SPLIT (N = 32): wave w -> column tile (w & 1), n-tiles (w >> 1) + 2j; PAIRED
    // (N >= 64): wave w -> n-tiles w + 4j for both column tiles (each weight fragment feeds two
    // MFMA chains). Accumulators start from the bias, or for cond layers from TPC / TPU.
    template <int l>
    static MPCD_DEV void hidden(const WFrag3<A::K[l], A::N[l], mode_for<A::N[l], R, W>()> &f, char *lds, int wave, int lane)
    {
        constexpr int K = A::K[l], N = A::N[l], MODE = mode_for<N, R, W>(), EPI = epi_of(l);
        using F = WFrag3<K, N, MODE>;
        constexpr int T = F::T, KC = F::KC;
        constexpr int NCT = MODE == SPLIT ? 1 : 2;
        static_assert(MODE == SPLIT || N % 64 == 0, "PAIRED layers need N % 64 == 0");
        const int col = lane & 15, q = lane >> 4;
        const bool in_shared = l == 0 && NB == 2;  // CFG: both branches read the candidate's x

        // activation fragments of both column tiles over the whole K, read up front
        u32x4 x[NCT][KC][3];
#pragma unroll
        for (int c = 0; c < NCT; ++c) {
            const int ct = MODE == SPLIT ? (wave & 1) : c;
            const int row = in_shared ? col : ct * 16 + col;
#pragma unroll
            for (int kc = 0; kc < KC; ++kc)
                load_x3(x[c][kc], lds + L::in_off(l) + row * L::in_rs(l) + (kc * 32 + 8 * q) * 2, L::in_pl(l));
        }
        f32x4 acc[T][NCT];
#pragma unroll
        for (int c = 0; c < NCT; ++c) {
            const int ct = MODE == SPLIT ? (wave & 1) : c;
            const float *init = reinterpret_cast<const float *>(
                lds + (EPI == EPI_CMISH ? ((NB == 2 && ct == 1) ? L::TPU : L::TPC) + cond_off(l / 2) * 4
                                        : L::BI + A::boff(l) * 4));
#pragma unroll
            for (int j = 0; j < T; ++j)
                acc[j][c] = *reinterpret_cast<const f32x4 *>(init + ntile_of<K, N, MODE>(wave, j) * 16 + 4 * q);
        }
        // Output tiles in G groups (T = 2: the n-tiles; else the column tiles); group g's MFMAs are
        // issued together with group g-1's epilogue: a bf16 MFMA leaves the SIMD's vector issue free
        // for 8 of its 16 cycles (unlike the f32 MFMA), so the Mish / split VALU rides in its shadow.
        constexpr bool BYJ = T == 2;
        constexpr int G = BYJ ? T : NCT;
        auto tile_mfma = [&](int j, int c) {
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) acc[j][c] = mfma_x3(f.v[j][kc], x[c][kc], acc[j][c]);
        };
        auto tile_epi = [&](int j, int c) {
            const int ct = MODE == SPLIT ? (wave & 1) : c;
            const int n = ntile_of<K, N, MODE>(wave, j) * 16 + 4 * q;
            f32x4 v = acc[j][c];
            if (EPI != EPI_NONE) {
                v.x = mish_scalar(v.x);
                v.y = mish_scalar(v.y);
                v.z = mish_scalar(v.z);
                v.w = mish_scalar(v.w);
            }
            u32x2 p0, p1, p2;
            split3(v, p0, p1, p2);
            char *o = lds + L::out_off(l) + (ct * 16 + col) * L::out_rs(l) + n * 2;
            *reinterpret_cast<u32x2 *>(o) = p0;
            *reinterpret_cast<u32x2 *>(o + L::out_pl(l)) = p1;
            *reinterpret_cast<u32x2 *>(o + 2 * L::out_pl(l)) = p2;
        };
        auto group = [&](int g, bool epi) {
#pragma unroll
            for (int i = 0; i < (BYJ ? NCT : 1); ++i) {
                const int j = BYJ ? g : 0, c = BYJ ? i : g;
                if (epi) tile_epi(j, c); else tile_mfma(j, c);
            }
        };
        // MFMAs per group, and ~3 VALU of the previous group's epilogue per MFMA
        constexpr int NM = (BYJ ? NCT : 1) * KC * 6;
        group(0, false);
#pragma unroll
        for (int g = 1; g < G; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            group(g, false);
            group(g - 1, true);
#pragma unroll
            for (int i = 0; i < NM; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // 3 VALU
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        group(G - 1, true);
    }

    // Hidden layer l on 8 waves (PAIR8 / WIDE8 above). Activation fragments are read one k-chunk
    // ahead rather than all up front (the partner wave covers the LDS latency), which keeps the
    // register budget of two waves per SIMD.
    template <int l>
    static MPCD_DEV void hidden8(const WFrag3<A::K[l], A::N[l], mode_for<A::N[l], R, W>()> &f, char *lds, int wave, int lane)
    {
        constexpr int K = A::K[l], N = A::N[l], MODE = mode_for<N, R, W>(), EPI = epi_of(l);
        using F = WFrag3<K, N, MODE>;
        constexpr int T = F::T, KC = F::KC, NT = N / 16;
        constexpr bool PR = MODE == PAIR8 || MODE == PAIRED;  // every column tile in each wave
        constexpr int NCT = PR ? R / 16 : 1;
        static_assert(PR || MODE == WIDE8, "8-wave layer modes, or PAIRED on 4 waves");
        const int col = lane & 15, q = lane >> 4;
        const bool in_shared = l == 0 && NB == 2;  // CFG: both branches read the candidate's x
        auto ct_of = [&](int c) { return PR ? c : (wave >> 2); };
        bool ok[T];
#pragma unroll
        for (int j = 0; j < T; ++j) ok[j] = ntile_of<K, N, MODE>(wave, j) < NT;
        f32x4 acc[T][NCT];
#pragma unroll
        for (int c = 0; c < NCT; ++c) {
            const int ct = ct_of(c);
            const float *init = reinterpret_cast<const float *>(
                lds + (EPI == EPI_CMISH ? (masked_of(ct, col) ? L::TPU : L::TPC) + cond_off(l / 2) * 4
                                        : L::BI + A::boff(l) * 4));
#pragma unroll
            for (int j = 0; j < T; ++j)
                acc[j][c] = *reinterpret_cast<const f32x4 *>(init + min(ntile_of<K, N, MODE>(wave, j), NT - 1) * 16 + 4 * q);
        }
        auto epi_tile = [&](int j, int c) {
            const int n = ntile_of<K, N, MODE>(wave, j) * 16 + 4 * q;
            f32x4 v = acc[j][c];
            if (EPI != EPI_NONE) {
                v.x = mish_scalar(v.x);
                v.y = mish_scalar(v.y);
                v.z = mish_scalar(v.z);
                v.w = mish_scalar(v.w);
            }
            u32x2 p0, p1, p2;
            split3(v, p0, p1, p2);
            char *o = lds + L::out_off(l) + (ct_of(c) * 16 + col) * L::out_rs(l) + n * 2;
            *reinterpret_cast<u32x2 *>(o) = p0;
            *reinterpret_cast<u32x2 *>(o + L::out_pl(l)) = p1;
            *reinterpret_cast<u32x2 *>(o + 2 * L::out_pl(l)) = p2;
        };
#if MPCD_X3_ILV
        if constexpr (PR && NCT == 2 && T == 1 && !(l == 0 && NB == 2)) {
            // One n-tile, two column tiles (the N = 128 layers at 32 rows): column tile 0's chain first,
            // then column tile 1's MFMAs with column tile 0's Mish / split / LDS stores scheduled in their
            // shadow (a bf16 MFMA leaves vector issue free for 8 of its 16 cycles), 3 VALU per MFMA.
            // Each weight fragment still feeds both column tiles from registers.
            auto ldx1 = [&](u32x4 (&x)[3], int c, int kc) {
                load_x3(x, lds + L::in_off(l) + (c * 16 + col) * L::in_rs(l) + (kc * 32 + 8 * q) * 2, L::in_pl(l));
            };
            auto chain = [&](int c) {
#if MPCD_X3_XALL
                // every k-chunk's fragments first: one LDS round trip per chain instead of one per chunk
                u32x4 xk[KC][3];
#pragma unroll
                for (int kc = 0; kc < KC; ++kc) ldx1(xk[kc], c, kc);
#pragma unroll
                for (int kc = 0; kc < KC; ++kc) acc[0][c] = mfma_x3(f.v[0][kc], xk[kc], acc[0][c]);
#else
                u32x4 xa[3], xb[3];
                ldx1(xa, c, 0);
#pragma unroll
                for (int kc = 0; kc < KC; ++kc) {
                    if (kc + 1 < KC) ldx1((kc & 1) ? xa : xb, c, kc + 1);
                    acc[0][c] = mfma_x3(f.v[0][kc], (kc & 1) ? xb : xa, acc[0][c]);
                }
#endif
            };
            chain(0);
            __builtin_amdgcn_sched_barrier(0);
            chain(1);
            epi_tile(0, 0);
#pragma unroll
            for (int i = 0; i < KC * 6; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // 3 VALU
            }
            __builtin_amdgcn_sched_barrier(0);
            epi_tile(0, 1);
            return;
        }
#endif
        auto ldx = [&](u32x4 (&x)[NCT][3], int kc) {
#pragma unroll
            for (int c = 0; c < NCT; ++c) {
                const int row = in_shared ? cand_of(ct_of(c), col) : ct_of(c) * 16 + col;
                load_x3(x[c], lds + L::in_off(l) + row * L::in_rs(l) + (kc * 32 + 8 * q) * 2, L::in_pl(l));
            }
        };
        u32x4 xc[NCT][3], xn[NCT][3];
        ldx(xc, 0);
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            if (kc + 1 < KC) ldx(xn, kc + 1);
#pragma unroll
            for (int j = 0; j < T; ++j)
                if (ok[j])
#pragma unroll
                    for (int c = 0; c < NCT; ++c) acc[j][c] = mfma_x3(f.v[j][kc], xc[c], acc[j][c]);
            if (kc + 1 < KC)
#pragma unroll
                for (int c = 0; c < NCT; ++c)
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl) xc[c][pl] = xn[c][pl];
        }
#pragma unroll
        for (int j = 0; j < T; ++j) {
            if (!ok[j]) continue;
#pragma unroll
            for (int c = 0; c < NCT; ++c) epi_tile(j, c);
        }
    }

    template <int l>
    static MPCD_DEV void layer(const WLoad<A::K[l], A::N[l], mode_for<A::N[l], R, W>()> &wl, char *lds, int wave, int lane)
    {
        WFrag3<A::K[l], A::N[l], mode_for<A::N[l], R, W>()> f;
        to_planes(wl, f);
        if constexpr (H8) hidden8<l>(f, lds, wave, lane);
        else hidden<l>(f, lds, wave, lane);
    }

    // x (4 features) -> fp32 row in XB and the three bf16 planes layer 0 reads
    static MPCD_DEV void store_x(char *lds, int cl, int n, const f32x4 &x)
    {
        *reinterpret_cast<f32x4 *>(lds + L::XB + (cl * L::SX + n) * 4) = x;
        u32x2 p0, p1, p2;
        split3(x, p0, p1, p2);
        char *o = lds + L::S1 + cl * L::RS + n * 2;
        *reinterpret_cast<u32x2 *>(o) = p0;
        *reinterpret_cast<u32x2 *>(o + L::PL) = p1;
        *reinterpret_cast<u32x2 *>(o + 2 * L::PL) = p2;
    }

    // final Linear (32 -> D0) + the denoise update (reference op order, see mlp_sampler.hip)
    static MPCD_DEV void final_and_update(const FW &f, char *lds, const MlpSampleArgs &p, const StepPlan &sp, int s,
                                          int64_t cand0, const f32x4 (&nz)[NZT][NB], uint32_t (&am)[2], int wave,
                                          int lane)
    {
        constexpr int T = FW::T, NT = D0 / 16;
        const int col = lane & 15, q = lane >> 4;
        const float *bias = reinterpret_cast<const float *>(lds + L::BI + A::boff(13) * 4);
        constexpr int NCT = R / 16;  // column tiles
        f32x4 acc[T][2];
#pragma unroll
        for (int j = 0; j < T; ++j) {  // idle tiles (D0 = 32, waves 2-3) read n-tile 0, unused
            const int nt = (NT % 4 == 0 || wave + 4 * j < NT) ? wave + 4 * j : 0;
            acc[j][0] = acc[j][1] = *reinterpret_cast<const f32x4 *>(bias + nt * 16 + 4 * q);
        }
#pragma unroll
        for (int c = 0; c < NCT; ++c) {
            u32x4 x[3];
            load_x3(x, lds + L::T1 + (c * 16 + col) * L::RS + 8 * q * 2, L::PL);
#pragma unroll
            for (int j = 0; j < T; ++j)
                if (NT % 4 == 0 || wave + 4 * j < NT) acc[j][c] = mfma_x3(f.v[j][0], x, acc[j][c]);
        }
        if (R == 16 && NB == 2) {
            // column c holds candidate c & 7's context row (c < 8) or masked row (c >= 8): bring the masked
            // row's eps next to the context row's (DPP row_ror:8 swaps the two halves of each 16-lane row)
#pragma unroll
            for (int j = 0; j < T; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    // element to a scalar first: clang lowers __builtin_bit_cast of an ext-vector element
                    // lvalue as a read of element 0
                    const float e = acc[j][0][r];
                    acc[j][1][r] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                        0, __builtin_bit_cast(int, e), 0x128, 0xF, 0xF, false));
                }
            if (col >= 8) return;  // lanes of the masked rows: their eps went to lane col - 8
        }
        const bool last = s == p.n_steps - 1;
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const int nt = wave + 4 * j;
            if (NT % 4 != 0 && nt >= NT) continue;
            const int n = nt * 16 + 4 * q;
#pragma unroll
            for (int g = 0; g < (NB == 2 ? 1 : NCT); ++g) {
                // NB == 2: one candidate per lane column, eps_c = tile 0, eps_u = tile 1 (R = 16: the DPP swap)
                // NB == 1: column tile g holds candidates 16g..16g+15
                const int cl = NB == 2 ? col : g * 16 + col;
                const f32x4 ec = acc[j][NB == 2 ? 0 : g];
                const f32x4 eu = acc[j][1];
                const int64_t gc = cand0 + cl;
                if (SMODE == MODE_EPS || SMODE == MODE_EPS1) {
                    if (gc < p.batch) {
                        *reinterpret_cast<f32x4 *>(p.x_out + (size_t)gc * D0 + n) = ec;
                        if (SMODE == MODE_EPS) *reinterpret_cast<f32x4 *>(p.chain + (size_t)gc * D0 + n) = eu;
                    }
                    continue;
                }
                const f32x4 x = *reinterpret_cast<const f32x4 *>(lds + L::XB + (cl * L::SX + n) * 4);
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
                    // chain |x| maximum: the x read here is x_T at s = 0 and every later slice; xn adds x_0
                    am[g] = max(am[g], max(abs_bits(xv), abs_bits(o)));
                }
                store_x(lds, cl, n, xn);
                if (gc < p.batch) {
                    if (p.chain) *reinterpret_cast<f32x4 *>(p.chain + ((size_t)(s + 1) * p.batch + gc) * D0 + n) = xn;
                    if (last) *reinterpret_cast<f32x4 *>(p.x_out + (size_t)gc * D0 + n) = xn;
                }
            }
        }
    }

    // noise of step s (slice s+1) for this lane's quads, fetched one step ahead of use
    static MPCD_DEV void fetch_noise(f32x4 (&nz)[NZT][NB], const MlpSampleArgs &p, const StepPlan &sp, int s,
                                     int64_t cand0, int wave, int lane)
    {
        constexpr int NT = D0 / 16;
#pragma unroll
        for (int j = 0; j < NZT; ++j)
#pragma unroll
            for (int g = 0; g < NB; ++g) nz[j][g] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (!IS_DDPM || !(sp.flags & PLAN_NOISE)) return;  // DDIM: sigma = 0
        const int col = lane & 15, q = lane >> 4;
#pragma unroll
        for (int j = 0; j < NZT; ++j) {
            const int nt = wave + 4 * j;
            if (NT % 4 != 0 && nt >= NT) continue;
            const int n = nt * 16 + 4 * q;
            const int64_t gc = cand0 + col;  // DDPM-CFG: NB == 2, one candidate per column (R = 16: columns < 8)
            if (gc >= p.batch || (R == 16 && col >= 8)) continue;
            if (SMODE == MODE_DDPM_XN)
                nz[j][0] = *reinterpret_cast<const f32x4 *>(p.noise + ((size_t)(s + 1) * p.batch + gc) * D0 + n);
            else
                nz[j][0] = philox_normal4(p.seed, (uint64_t)(p.global_offset + gc), (uint32_t)(s + 1), (uint32_t)(n >> 2));
        }
    }

    static MPCD_DEV void run(const MlpSampleArgs &p)
    {
        extern __shared__ float lds_f[];
        char *lds = reinterpret_cast<char *>(lds_f);
        const int lane = threadIdx.x & 63;
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const int64_t cand0 = (int64_t)blockIdx.x * CPW;
        int lane16 = lane * 16;
        const float *wp = p.wpack;
        int wofs = 0;
        auto wptr = [&](int l) { return wp + wofs + woffx<D0>(l); };
        float *bi = reinterpret_cast<float *>(lds + L::BI);
        float *bic = reinterpret_cast<float *>(lds + L::BIC);
        float *cps = reinterpret_cast<float *>(lds + L::CPS);

        for (int l = 0; l < NLAYER; ++l)
            for (int i = threadIdx.x; i < A::N[l]; i += NTHR) bi[A::boff(l) + i] = wp[woffx<D0>(l) + wfl<D0>(l) + i];
        for (int j = 0; j < 6; ++j)
            for (int i = threadIdx.x; i < A::N[2 * j + 1]; i += NTHR)
                bic[cond_off(j) + i] = wp[woffx<D0>(2 * j + 1) + wfl<D0>(2 * j + 1) + i];
        for (int i = threadIdx.x; i < COND_TOTAL; i += NTHR)  // ctx_fused: as mlp_rw.hip
            cps[i] = !CTX ? 0.f
                          : p.ctx_fused ? ctx_proj_col(p.ctx_row, p.ctx_dim, p.cond_layers, p.n_cond, p.cond_dim, i)
                                        : p.cproj[i];
        if (threadIdx.x < CPW) reinterpret_cast<uint32_t *>(lds + L::AMX)[threadIdx.x] = 0u;
        uint32_t am[2] = {0u, 0u};
        // x_T (fp32 + planes)
        for (int i = threadIdx.x; i < CPW * QUADS; i += NTHR) {
            const int c = i / QUADS, qd = i - c * QUADS;
            const int64_t gc = cand0 + c;
            f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
            if (gc < p.batch) {
                z = p.noise ? *reinterpret_cast<const f32x4 *>(p.noise + (size_t)gc * D0 + qd * 4)
                            : philox_normal4(p.seed, (uint64_t)(p.global_offset + gc), 0u, (uint32_t)qd);
                if (p.chain && SMODE != MODE_EPS) *reinterpret_cast<f32x4 *>(p.chain + (size_t)gc * D0 + qd * 4) = z;
            }
            store_x(lds, c, qd * 4, z);
        }

        WLoad<A::K[0], A::N[0], mode_for<A::N[0], R, W>()> w0;
        load_w3(w0, wptr(0), wave, lane16);
        f32x4 nz[NZT][NB];
        StepPlan sp = load_plan(p.plan, 0);
        if (wave < 4) fetch_noise(nz, p, sp, 0, cand0, wave, lane);
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
            // launder the weight base: stops LICM hoisting every layer's weight loads out of the loop
            asm volatile("" : "+s"(wofs), "+v"(lane16));
            WLoad<A::K[1], A::N[1], mode_for<A::N[1], R, W>()> w1;
            load_w3(w1, wptr(1), wave, lane16);
            bar(0);
            // this step's time projections + cond biases (+ shared context part) -> TPU / TPC
            if (threadIdx.x < COND_TOTAL / 4) {
                const f32x4 u = tpre + reinterpret_cast<const f32x4 *>(lds + L::BIC)[tpi];
                reinterpret_cast<f32x4 *>(lds + L::TPU)[tpi] = u;
                reinterpret_cast<f32x4 *>(lds + L::TPC)[tpi] = u + reinterpret_cast<const f32x4 *>(lds + L::CPS)[tpi];
            }
            tpre = reinterpret_cast<const f32x4 *>(p.tproj + (size_t)(s + 1 < p.n_steps ? s + 1 : s) * COND_TOTAL)[tpi];
            layer<0>(w0, lds, wave, lane);
            WLoad<A::K[2], A::N[2], mode_for<A::N[2], R, W>()> w2;
            load_w3(w2, wptr(2), wave, lane16);
            bar(1);
            layer<1>(w1, lds, wave, lane);
            WLoad<A::K[3], A::N[3], mode_for<A::N[3], R, W>()> w3;
            load_w3(w3, wptr(3), wave, lane16);
            bar(2);
            layer<2>(w2, lds, wave, lane);
            WLoad<A::K[4], A::N[4], mode_for<A::N[4], R, W>()> w4;
            load_w3(w4, wptr(4), wave, lane16);
            bar(3);
            layer<3>(w3, lds, wave, lane);
            WLoad<A::K[5], A::N[5], mode_for<A::N[5], R, W>()> w5;
            load_w3(w5, wptr(5), wave, lane16);
            WLoad<A::K[6], A::N[6], mode_for<A::N[6], R, W>()> w6;
#if MPCD_X3_LEAD2  // the 128-wide layers' weights two segments ahead (their L2 latency outlasts one segment)
            load_w3(w6, wptr(6), wave, lane16);
#endif
            bar(4);
            layer<4>(w4, lds, wave, lane);
            WLoad<A::K[7], A::N[7], mode_for<A::N[7], R, W>()> w7;
#if MPCD_X3_LEAD2
            load_w3(w7, wptr(7), wave, lane16);
#else
            load_w3(w6, wptr(6), wave, lane16);
#endif
            bar(5);
            layer<5>(w5, lds, wave, lane);
#if !MPCD_X3_LEAD2
            load_w3(w7, wptr(7), wave, lane16);
#endif
            bar(6);
            layer<6>(w6, lds, wave, lane);
            WLoad<A::K[8], A::N[8], mode_for<A::N[8], R, W>()> w8;
            load_w3(w8, wptr(8), wave, lane16);
            bar(7);
            layer<7>(w7, lds, wave, lane);
            WLoad<A::K[9], A::N[9], mode_for<A::N[9], R, W>()> w9;
            load_w3(w9, wptr(9), wave, lane16);
            bar(8);
            layer<8>(w8, lds, wave, lane);
            WLoad<A::K[10], A::N[10], mode_for<A::N[10], R, W>()> w10;
            load_w3(w10, wptr(10), wave, lane16);
            bar(9);
            layer<9>(w9, lds, wave, lane);
            WLoad<A::K[11], A::N[11], mode_for<A::N[11], R, W>()> w11;
            load_w3(w11, wptr(11), wave, lane16);
            bar(10);
            layer<10>(w10, lds, wave, lane);
            WLoad<A::K[12], A::N[12], mode_for<A::N[12], R, W>()> w12;
            load_w3(w12, wptr(12), wave, lane16);
            bar(11);
            layer<11>(w11, lds, wave, lane);
            FWL w13;
            load_w3(w13, wptr(13), wave, lane16, wave < 4);
            bar(12);
            layer<12>(w12, lds, wave, lane);
            const StepPlan cur = sp;
            f32x4 nzc[NZT][NB];
#pragma unroll
            for (int j = 0; j < NZT; ++j)
#pragma unroll
                for (int g = 0; g < NB; ++g) nzc[j][g] = nz[j][g];
            if (s + 1 < p.n_steps) {
                sp = load_plan(p.plan, s + 1);
                if (wave < 4) fetch_noise(nz, p, sp, s + 1, cand0, wave, lane);
            }
            // next step's layer-0 weights; unconditional (a path-dependent load count drains vmcnt(0))
            load_w3(w0, wptr(0), wave, lane16);
            bar(13);
            if (wave < 4) {
                FW f13;
                to_planes(w13, f13);
                final_and_update(f13, lds, p, cur, s, cand0, nzc, am, wave, lane);
            }
        }
        if (SMODE != MODE_EPS && SMODE != MODE_EPS1 && p.chain_absmax) {
            const int col = lane & 15;
            store_chain_absmax<CPW, NTHR>(reinterpret_cast<uint32_t *>(lds + L::AMX), am, col,
                                             (NB == 2 || R == 16) ? -1 : 16 + col,
                                             wave < 4 && (NB == 1 || R == 32 || col < 8), p.chain_absmax, cand0, p.batch);
        }
#ifdef MPCD_PROF_LAYERS
        {
            const uint64_t t = __builtin_readcyclecounter();
            tacc[2 * 15] += t - tprev;
            if (p.dbg && blockIdx.x < 32 / W && lane == 0)  // 32 wave slots
                for (int i = 0; i < 32; ++i) p.dbg[(blockIdx.x * W + (threadIdx.x >> 6)) * 32 + i] = (float)tacc[i];
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

// (R, W) = (16, 4): 256 threads, two workgroups per CU (two waves per SIMD from independent workgroups)
template <int D0, int SMODE, bool CTX, int R, int W>
__global__ __launch_bounds__(64 * W, W == 4 ? 2 : 1) void mlp_x3_kernel(const MlpSampleArgs p)
{
    MlpX3<D0, SMODE, CTX, R, W>::run(p);
}

template <int D0, int SMODE, bool CTX, int R, int W>
hipError_t launch_x3_r(const MlpSampleArgs &a, hipStream_t stream)
{
    using L = Lds3<D0, MlpX3<D0, SMODE, CTX, R, W>::NB, R>;
    static_assert(W == 8 || 2 * L::total <= 160 * 1024, "two 4-wave workgroups per CU");
    static_assert(L::total <= 160 * 1024, "LDS budget (160 KiB per CU)");
    if (hipError_t e = allow_max_lds<&mlp_x3_kernel<D0, SMODE, CTX, R, W>>(); e != hipSuccess) return e;
    const int64_t blocks = (a.batch + L::CPW - 1) / L::CPW;
    return launch_sampler_kernel(mlp_x3_kernel<D0, SMODE, CTX, R, W>, dim3((unsigned)blocks), dim3(64 * W), (size_t)L::total, stream, a);
}

// Workgroup layout (rows x waves): 32x8 (one per CU), 16x8 when 32-row workgroups would leave CUs idle
// (fewer than one per CU), 16x4 = two independent 4-wave workgroups per CU, whose barriers and
// latency chains interleave on each SIMD instead of coinciding. MPCD_MLP_LAYOUT=32x8|16x8|16x4 forces.
// rw32 / rw16: mlp_rw.hip (4 waves, the 128-wide layers' weights resident in registers), 32 or 16 rows.
enum { LAYOUT_32x8 = 0, LAYOUT_16x8 = 1, LAYOUT_16x4 = 2, LAYOUT_RW32 = 3, LAYOUT_RW16 = 4 };
std::atomic<int> g_force_layout{-1};  // mpcd_mlp_force_layout (tests: every layout against the oracle)
int mlp_x3_layout(int64_t batch, int nb)
{
    if (const int f = g_force_layout.load(); f >= 0) return f;
    static const int forced = [] {
        const char *e = getenv("MPCD_MLP_LAYOUT");
        if (!e || !e[0]) return -1;
        return !strcmp(e, "32x8") ? (int)LAYOUT_32x8 : !strcmp(e, "16x8") ? (int)LAYOUT_16x8 : !strcmp(e, "16x4") ? (int)LAYOUT_16x4
             : !strcmp(e, "rw32") ? (int)LAYOUT_RW32 : !strcmp(e, "rw16") ? (int)LAYOUT_RW16 : -1;
    }();
    if (forced >= 0) return forced;
    // the resident-weight kernel (mlp_rw.hip) at every batch: 32-row workgroups (cfg2: 1.187 vs 1.252 ms kernel for
    // the streaming 32x8), 16-row ones below one 32-row workgroup per CU (the 512-candidate strong-scaling shard:
    // 0.87 vs 1.04 ms per control step for 16x8; cfg1 0.41 vs 0.49 ms kernel) - profiles/r4_mlp_layouts.txt
    const int n_cu = device_cu_count();
    return (batch * nb + 31) / 32 < n_cu ? LAYOUT_RW16 : LAYOUT_RW32;
}

template <int D0, int SMODE, bool CTX>
hipError_t launch_x3(const MlpSampleArgs &a, int layout, hipStream_t stream)
{
    constexpr int NB = MlpX3<D0, SMODE, CTX, 32>::NB;
    switch (layout) {
    case LAYOUT_16x8: return launch_x3_r<D0, SMODE, CTX, 16, 8>(a, stream);
    case LAYOUT_16x4:  // where two 16-row workgroups fit the CU's LDS (else 16x8)
        if constexpr (2 * Lds3<D0, NB, 16>::total <= 160 * 1024) return launch_x3_r<D0, SMODE, CTX, 16, 4>(a, stream);
        else return launch_x3_r<D0, SMODE, CTX, 16, 8>(a, stream);
    default: return launch_x3_r<D0, SMODE, CTX, 32, WAVES>(a, stream);
    }
}

template <int D0>
hipError_t launch_x3_d0(const MlpSampleArgs &a, int lay, hipStream_t stream)
{
    const bool ctx = a.cproj != nullptr;
    switch (a.mode) {
    case MODE_DDPM_CFG:
        if (a.noise) return ctx ? launch_x3<D0, MODE_DDPM_XN, true>(a, lay, stream) : launch_x3<D0, MODE_DDPM_XN, false>(a, lay, stream);
        return ctx ? launch_x3<D0, MODE_DDPM_CFG, true>(a, lay, stream) : launch_x3<D0, MODE_DDPM_CFG, false>(a, lay, stream);
    case MODE_DDIM_CFG: return ctx ? launch_x3<D0, MODE_DDIM_CFG, true>(a, lay, stream) : launch_x3<D0, MODE_DDIM_CFG, false>(a, lay, stream);
    case MODE_DDIM: return ctx ? launch_x3<D0, MODE_DDIM, true>(a, lay, stream) : launch_x3<D0, MODE_DDIM, false>(a, lay, stream);
    case MODE_EPS: return ctx ? launch_x3<D0, MODE_EPS, true>(a, lay, stream) : launch_x3<D0, MODE_EPS, false>(a, lay, stream);
    case MODE_EPS1: return ctx ? launch_x3<D0, MODE_EPS1, true>(a, lay, stream) : launch_x3<D0, MODE_EPS1, false>(a, lay, stream);
    }
    return hipErrorInvalidValue;
}

}  // namespace

void mlp_x3_force_layout(int layout) { g_force_layout.store(layout); }
int mlp_x3_layout_of(int64_t batch, int nb) { return mlp_x3_layout(batch, nb); }

int mlp_packed_floats_x3(int d0)
{
    switch (d0) {
    case 32: return woffx<32>(NLAYER);
    case 64: return woffx<64>(NLAYER);
    case 128: return woffx<128>(NLAYER);
    default: return -1;
    }
}

// Split Linear l (torch weight [N][K]) into three bf16 planes (w = w0 + w1 + w2, round to nearest
// even at each level, remainders exact) and pack them as the MFMA A operand of
// v_mfma_f32_16x16x32_bf16: chunk (nt, kc, plane) = 64 lanes x 8 bf16, lane l holding
// W[nt*16 + (l&15)][kc*32 + 8*(l>>4) + j], j = 0..7; then the fp32 bias [N].
static uint16_t bf16_rne(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)(u >> 16);  // inf / nan: truncate
    const uint32_t r = u + 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(r >> 16);
}
static float bf16_val(uint16_t h)
{
    const uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

void mlp_pack_weights_x3(int d0, const float *const *lin_w, const float *const *lin_b, float *out)
{
    const int Ks[NLAYER] = {d0, 32, 32, 64, 64, 128, 128, 128, 256, 64, 128, 32, 32, 32};
    const int Ns[NLAYER] = {32, 32, 64, 64, 128, 128, 128, 128, 64, 64, 32, 32, 32, d0};
    size_t o = 0;  // in floats
    for (int l = 0; l < NLAYER; ++l) {
        const int K = Ks[l], N = Ns[l], KC = K / 32, NT = N / 16;
        uint16_t *pk = reinterpret_cast<uint16_t *>(out + o);
        for (int nt = 0; nt < NT; ++nt)
            for (int kc = 0; kc < KC; ++kc)
                for (int lane = 0; lane < 64; ++lane)
                    for (int j = 0; j < 8; ++j) {
                        const float w = lin_w[l][(size_t)(nt * 16 + (lane & 15)) * K + kc * 32 + 8 * (lane >> 4) + j];
                        if (WPL == 2) {  // fp32 as loaded; the kernel splits it (to_planes)
                            out[o + ((size_t)(nt * KC + kc) * 64 + lane) * 8 + j] = w;
                            continue;
                        }
                        const uint16_t h0 = bf16_rne(w);
                        const float r1 = w - bf16_val(h0);
                        const uint16_t h1 = bf16_rne(r1);
                        const float r2 = r1 - bf16_val(h1);
                        const uint16_t h2 = bf16_rne(r2);
                        const uint16_t hs[3] = {h0, h1, h2};
                        for (int pl = 0; pl < 3; ++pl)
                            pk[(((size_t)(nt * KC + kc) * 3 + pl) * 64 + lane) * 8 + j] = hs[pl];
                    }
        o += (size_t)WPL * K * N / 2;
        for (int n = 0; n < N; ++n) out[o + n] = lin_b[l][n];
        o += N;
    }
}

hipError_t launch_mlp_x3(int d0, int nb, const MlpSampleArgs &a, hipStream_t stream)
{
    if ((nb == 1) != (a.mode == MODE_DDIM || a.mode == MODE_EPS1)) return hipErrorInvalidValue;
    if (a.cproj && a.cproj_stride != 0) return hipErrorInvalidValue;  // shared context only
    const int lay = mlp_x3_layout(a.batch, nb);  // decided once per call
    if (lay == LAYOUT_RW32 || lay == LAYOUT_RW16) return launch_mlp_rw(d0, lay == LAYOUT_RW32 ? 32 : 16, a, stream);
    switch (d0) {
    case 32: return launch_x3_d0<32>(a, lay, stream);
    case 64: return launch_x3_d0<64>(a, lay, stream);
    case 128: return launch_x3_d0<128>(a, lay, stream);
    }
    return hipErrorInvalidValue;
}
