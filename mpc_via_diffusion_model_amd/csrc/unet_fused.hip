// The whole ConditionedTemporalUnet noise-net forward of one denoise step in ONE launch, activations in LDS.
//
// Reference: ConditionedTemporalUnet.forward (temporal_unet.py:287-358) with ResidualTemporalBlock,
// Conv1dBlock, Downsample1d, Upsample1d (layers.py:258-355), base 32, dim_mults (1, 2, 4); then the CFG
// denoise update of that step (p_mean_variance_CFG + ddpm_cart_pole_sample_fn, diffusion_model_base.py:
// 164-178, sample_functions.py:17-44; or the build-defined CFG-DDIM).
//
// A workgroup (8 waves, two per SIMD, one workgroup per CU) owns R rows = R/2 candidates x the two CFG
// branches (rows [0, R/2): context, [R/2, R): masked context) and runs all 35 convs of the net on them:
// every activation stays in LDS, channels-last [plane][row][position][channel] with zero halo positions,
// already split into the MFMA operand planes (three bf16 planes for MPCD_F32X3, one fp16 plane for
// MPCD_F16), so each conv's B operand is read straight from LDS with ds_read_b128 and its A operand
// (the packed weights, unet_pack_mx) streams from L2 by buffer loads a few k-chunks ahead. The only HBM
// traffic per step is x and the result (plus one skip tensor, h1, spilled to a scratch buffer while the
// lower levels run: it would not fit the LDS next to the others).
//
// Per conv (an op of the host-built program, FOp): implicit GEMM on v_mfma_f32_16x16x32_{f16,bf16} -
// wave w owns n-tile (w mod NT) and NC consecutive 16-column tiles of the R x L output columns (NC =
// R*H/64 or half that; the op table is built so every wave has the same work); the accumulators start
// from the bias; GroupNorm statistics come straight from the accumulators (shifted sums per 16-column
// segment, combined across segments in a fixed order with Chan's formula: deterministic, independent of
// the batch and of the workgroup); the epilogue (GroupNorm affine -> Mish -> + cond / + residual) runs in
// registers and writes the next conv's operand planes. Layer order, views and LDS placement: host side
// (unet_fused_prepare below).
#include <hip/hip_runtime.h>

#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "mx_common.h"
#include "unet.h"

namespace {

using namespace mx;

constexpr int FT = 512;  // threads per workgroup (8 waves)

struct FView {
    int32_t off;   // byte offset in plane 0 of (row 0, position 0, the view's first channel)
    int32_t cs;    // bytes per position
    int32_t rowB;  // bytes per row
    int32_t L, C;  // positions, channels
    int32_t hl, hr;  // zero halo positions left / right of each row
};

enum { FK_SAME5 = 0, FK_DOWN3 = 1, FK_UP4 = 2, FK_PW1 = 3, FK_RESTORE = 4 };
enum { FE_BIAS = 0, FE_GN = 1, FE_GN_COND = 2, FE_GN_RES = 3, FE_EPS = 4 };
static_assert(FK_SAME5 == UCONV_SAME5 && FK_DOWN3 == UCONV_DOWN3 && FK_UP4 == UCONV_UP4 && FK_PW1 == UCONV_PW1,
              "conv kinds");

struct FOp {
    const uint16_t *w;                  // packed A fragments [parity][n-tile][k-chunk][plane][64][8]
    const float *bias, *gnw, *gnb;
    int32_t kind, epi, cond_off, spill;  // spill: also write the output to the skip scratch (RESTORE: read it back)
    int32_t cinp, cpt_sh, kc, nt_sh;     // K per tap, log2 k-chunks per tap (-1: cinp 8 = 4 taps per chunk),
                                         // k-chunks, log2 n-tiles
    int32_t cout, lin, lout, lsh;        // lsh: log2 of the columns per row and parity (lout, or lin for UP4)
    int32_t half, cpg_sh, alias_in, pad;  // half: NC = NCB / 2; cpg_sh: log2 channels per GroupNorm group;
                                          // alias_in: the output overwrites the GEMM input
    FView in, res, out;
};

struct FArgs {
    const FOp *ops;
    int32_t n_ops, plb;       // ops; bytes per operand plane
    int32_t e_off, stat_off;  // LDS byte offsets: eps [R][H][d] fp32; GroupNorm partials + statistics
    FView xv;                 // staged x (8 channels, halo 2 / 5)
    float *x;                 // sampler state [B][H][d] (updated in place), or the input of MODE_EPS
    int64_t batch, goff;
    int32_t d, mode, clamp_x0, s, last, pad;
    const float *tp, *cp;     // tproj row of this step; cproj (per candidate or shared) or null
    int64_t cp_stride;
    const StepPlan *plan;
    float wp1, wf;
    const float *noise;
    uint64_t seed;
    float *chain, *x_out;
    uint32_t *amq;
    float *eps_c, *eps_u;     // MODE_EPS outputs
    char *scratch;            // skip spill: [row][L][C], fp16 (P = 1) or fp32 (P = 3)
};

constexpr int kGroups = 8;  // GroupNorm groups of every 32 / 64 / 128-channel conv (group_norm_n_groups)

template <int R, int H>
constexpr int part_floats() { return R * (H >= 16 ? H / 16 : 1) * kGroups * 4; }

// ---- one conv of the program: GEMM + statistics + epilogue, NC 16-column tiles per wave
template <int P, int R, int H, int NC, int KIND>
MPCD_DEV void conv_op(const FArgs &a, const FOp &op, int64_t cand0, int64_t row0)
{
    extern __shared__ __attribute__((aligned(16))) char sm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 15, q = lane >> 4;
    const int nt_sh = op.nt_sh, NT = 1 << nt_sh;
    const int nt = wave & (NT - 1), wc = wave >> nt_sh;
    const int t0 = wc * NC;  // this wave's first column tile
    const int plb = a.plb;

    // ---- columns of the wave's tiles: (row, output position) and the tap-0 input position
    int par = 0;
    if (KIND == FK_UP4) par = t0 >= ((R * op.lin) >> 4) ? 1 : 0;  // tiles per parity = R * lin / 16 (host: NC divides it)
    int bb[NC], cr[NC], co[NC];
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) {
        int c = (t0 + cc) * 16 + col;
        int r, o, pos0;
        if (KIND == FK_UP4) {
            c -= par * R * op.lin;
            r = c >> op.lsh;
            const int m = c & (op.lin - 1);
            pos0 = par ? m + 1 : m;  // slot s reads position pos0 - s (ConvTranspose1d k4 s2 p1)
            o = 2 * m + par;
        } else {
            r = c >> op.lsh;
            o = c & (op.lout - 1);
            pos0 = KIND == FK_SAME5 ? o - 2 : KIND == FK_DOWN3 ? 2 * o - 1 : o;
        }
        bb[cc] = op.in.off + r * op.in.rowB + pos0 * op.in.cs;
        cr[cc] = r;
        co[cc] = o;
    }

    // ---- implicit GEMM: acc[cc] (channels nt*16 + 4q + e, column tile t0 + cc)
    const int KC = op.kc;
    const int n0 = nt * 16 + 4 * q;
    f32x4 acc[NC];
    {
        f32x4 b;
#pragma unroll
        for (int e = 0; e < 4; ++e) b[e] = n0 + e < op.cout ? op.bias[n0 + e] : 0.f;
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) acc[cc] = b;
    }
    const int npar = KIND == FK_UP4 ? 2 : 1;
    const uint64_t wa = (uint64_t)op.w;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)wa, (short)0, (int)(npar * NT * KC * P * 1024), 0x00020000);
    const int lane16 = lane * 16;
    auto load_a = [&](u32x4 (&A)[P], int kc) {
#pragma unroll
        for (int pl = 0; pl < P; ++pl) {
            const int soff = __builtin_amdgcn_readfirstlane((((par * NT + nt) * KC + kc) * P + pl) * 1024);
            A[pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane16, soff, 0));
        }
    };
    const int cpt_sh = op.cpt_sh, ics = op.in.cs;
    auto koff = [&](int kc) -> int {
        int tap, ci;
        if (cpt_sh >= 0) {
            tap = kc >> cpt_sh;
            ci = ((kc & ((1 << cpt_sh) - 1)) << 5) + 8 * q;
        } else {  // 8 channels per tap: one chunk = 4 taps, lane quarter q takes tap 4kc + q
            tap = 4 * kc + q;
            ci = 0;
        }
        return (KIND == FK_UP4 ? -tap : tap) * ics + 2 * ci;
    };
    auto load_b = [&](u32x4 (&B)[NC][P], int ko) {
#pragma unroll
        for (int cc = 0; cc < NC; ++cc)
#pragma unroll
            for (int pl = 0; pl < P; ++pl) B[cc][pl] = *reinterpret_cast<const u32x4 *>(sm + bb[cc] + ko + pl * plb);
    };
    auto mmas = [&](const u32x4 (&A)[P], const u32x4 (&B)[NC][P]) {
#pragma unroll
        for (int i = 0; i < NPROD(P); ++i)
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) acc[cc] = mma<P>(A[PA<P>(i)], B[cc][PB<P>(i)], acc[cc]);
    };
    constexpr int DA = P == 1 ? 4 : 2;  // A chunks in flight (L2 latency)
    u32x4 A[DA][P];
#pragma unroll
    for (int s = 0; s < DA; ++s) load_a(A[s], min(s, KC - 1));
    u32x4 Bc[NC][P], Bn[NC][P];
    load_b(Bc, koff(0));
    int kc = 0;
    for (; kc + DA <= KC; kc += DA) {
#pragma unroll
        for (int s = 0; s < DA; ++s) {
            load_b(Bn, koff(min(kc + s + 1, KC - 1)));
            mmas(A[s], Bc);
            load_a(A[s], min(kc + s + DA, KC - 1));
#pragma unroll
            for (int cc = 0; cc < NC; ++cc)
#pragma unroll
                for (int pl = 0; pl < P; ++pl) Bc[cc][pl] = Bn[cc][pl];
        }
    }
#pragma unroll
    for (int s = 0; s < DA - 1; ++s) {  // tail: A[s] holds chunk kc + s
        if (kc + s < KC) {
            load_b(Bn, koff(min(kc + s + 1, KC - 1)));
            mmas(A[s], Bc);
#pragma unroll
            for (int cc = 0; cc < NC; ++cc)
#pragma unroll
                for (int pl = 0; pl < P; ++pl) Bc[cc][pl] = Bn[cc][pl];
        }
    }

    // ---- GroupNorm statistics from the accumulators
    const int epi = op.epi;
    const bool gn = epi == FE_GN || epi == FE_GN_COND || epi == FE_GN_RES;
    float *part = reinterpret_cast<float *>(sm + a.stat_off);  // [segment][group][S1, S2, shift, -]
    float *stat = part + part_floats<R, H>();                  // [row][group][mean, rstd]
    const int g = gn ? n0 >> op.cpg_sh : 0;
    if (gn) {
        const int L = op.lout, seg_len = L < 16 ? L : 16, seg_sh = L < 16 ? 3 : 4;
        const int qmask = (1 << (op.cpg_sh - 2)) - 1;  // lane quarters per group - 1: 0, 1 or 3
        const int src = (col & ~(seg_len - 1)) | ((q & ~qmask) << 4);
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) {
            // shift = the segment's first value of the group: the sums are of (x - shift) = O(std)
            const float sh = __shfl(acc[cc][0], src);
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float dv = acc[cc][e] - sh;
                s1 += dv;
                s2 += dv * dv;
            }
            for (int m = 1; m < seg_len; m <<= 1) {
                s1 += __shfl_xor(s1, m);
                s2 += __shfl_xor(s2, m);
            }
            if (qmask >= 1) {
                s1 += __shfl_xor(s1, 16);
                s2 += __shfl_xor(s2, 16);
            }
            if (qmask >= 3) {
                s1 += __shfl_xor(s1, 32);
                s2 += __shfl_xor(s2, 32);
            }
            if ((col & (seg_len - 1)) == 0 && (q & qmask) == 0) {
                const int seg = ((t0 + cc) * 16 + col) >> seg_sh;
                *reinterpret_cast<f32x4 *>(part + (seg * kGroups + g) * 4) = f32x4{s1, s2, sh, 0.f};
            }
        }
        __syncthreads();
        if (tid < R * kGroups) {  // one (row, group) per thread: its segments in order (Chan et al.)
            const int r = tid / kGroups, gg = tid - r * kGroups;
            const int nseg = L >> seg_sh;
            const double n1 = (double)(seg_len << op.cpg_sh);
            double n = 0.0, mean = 0.0, m2 = 0.0;
            for (int k = 0; k < nseg; ++k) {
                const f32x4 p = *reinterpret_cast<const f32x4 *>(part + ((r * nseg + k) * kGroups + gg) * 4);
                const double mk = (double)p[2] + (double)p[0] / n1;
                const double m2k = (double)p[1] - (double)p[0] * (double)p[0] / n1;
                const double nn = n + n1, dl = mk - mean;
                mean += dl * (n1 / nn);
                m2 += m2k + dl * dl * (n * n1 / nn);
                n = nn;
            }
            const double var = fmax(m2 / n, 0.0);
            stat[2 * tid] = (float)mean;
            stat[2 * tid + 1] = (float)(1.0 / sqrt(var + 1e-5));
        }
        __syncthreads();
    } else if (op.alias_in) {
        __syncthreads();
    }

    // ---- epilogue: GroupNorm affine -> Mish -> + cond / + residual, written as the next conv's planes
    f32x4 gw = {0.f, 0.f, 0.f, 0.f}, gb = gw, cv0 = gw, cv1 = gw;
    if (gn) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // GroupNorm affine: parameter-blob offsets need not be 16-byte aligned
            gw[e] = op.gnw[n0 + e];
            gb[e] = op.gnb[n0 + e];
        }
        if (epi == FE_GN_COND) {
            cv1 = ldg4(a.tp + op.cond_off + n0);  // masked branch: Linear(Mish(cat(t_emb, 0))) = the time part
            cv0 = (a.cp && !a.cp_stride) ? cv1 + ldg4(a.cp + op.cond_off + n0) : cv1;
        }
    }
    float *E = reinterpret_cast<float *>(sm + a.e_off);
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) {
        const int r = cr[cc], o = co[cc];
        f32x4 v = acc[cc];
        if (gn) {
            const float mean = stat[2 * (r * kGroups + g)], rstd = stat[2 * (r * kGroups + g) + 1];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float scale = rstd * gw[e];
                const float shift = -scale * mean + gb[e];
                v[e] = mish(v[e] * scale + shift);
            }
            if (epi == FE_GN_COND) {
                const bool masked = r >= R / 2;
                f32x4 cv = masked ? cv1 : cv0;
                if (!masked && a.cp && a.cp_stride) {
                    const int64_t cand = cand0 + r;
                    if (cand < a.batch) cv = cv + ldg4(a.cp + (size_t)cand * a.cp_stride + op.cond_off + n0);
                }
                v = v + cv;
            } else if (epi == FE_GN_RES) {
                u32x2 pr[P];
                const char *s = sm + op.res.off + r * op.res.rowB + o * op.res.cs + 2 * n0;
#pragma unroll
                for (int pl = 0; pl < P; ++pl) pr[pl] = *reinterpret_cast<const u32x2 *>(s + pl * plb);
                v = v + join4<P>(pr);
            }
        }
        if (epi == FE_EPS) {  // the net's output (cout = d): fp32 for the update
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (n0 + e < op.cout) E[(r * H + o) * op.cout + n0 + e] = v[e];
            continue;
        }
        u32x2 pk[P];
        split4<P>(v, pk);
        char *dst = sm + op.out.off + r * op.out.rowB + o * op.out.cs + 2 * n0;
#pragma unroll
        for (int pl = 0; pl < P; ++pl) *reinterpret_cast<u32x2 *>(dst + pl * plb) = pk[pl];
        if (op.spill) {  // the skip tensor, as the LDS holds it (fp16), or its fp32 value (re-split on restore)
            const size_t e = ((size_t)(row0 + r) * op.out.L + o) * op.out.C + n0;
            if constexpr (P == 1)
                *reinterpret_cast<u32x2 *>(a.scratch + 2 * e) = pk[0];
            else
                *reinterpret_cast<f32x4 *>(a.scratch + 4 * e) = v;
        }
    }
}

// zero halo positions of a view (every row, every plane, the view's channels)
template <int P, int R>
MPCD_DEV void zero_halo(const FView &v, int plb)
{
    extern __shared__ __attribute__((aligned(16))) char sm[];
    const int hp = v.hl + v.hr, u = v.C >> 3;  // 16-byte units per position
    const int n = P * R * hp * u;
    for (int i = threadIdx.x; i < n; i += FT) {
        const int k = i % u, t = i / u, h = t % hp, rp = t / hp, r = rp % R, pl = rp / R;
        const int pos = h < v.hl ? h - v.hl : v.L + h - v.hl;
        *reinterpret_cast<u32x4 *>(sm + v.off + pl * plb + r * v.rowB + pos * v.cs + 16 * k) = u32x4{0u, 0u, 0u, 0u};
    }
}

// skip tensor back from the scratch into its LDS view
template <int P, int R>
MPCD_DEV void restore_op(const FArgs &a, const FOp &op, int64_t row0)
{
    extern __shared__ __attribute__((aligned(16))) char sm[];
    const FView &v = op.out;
    const int u = v.C >> 3, n = R * v.L * u;
    for (int i = threadIdx.x; i < n; i += FT) {
        const int k = i % u, t = i / u, p = t % v.L, r = t / v.L;
        const size_t e = ((size_t)(row0 + r) * v.L + p) * v.C + 8 * k;
        char *dst = sm + v.off + r * v.rowB + p * v.cs + 16 * k;
        if constexpr (P == 1) {
            *reinterpret_cast<u32x4 *>(dst) = __builtin_bit_cast(u32x4, ldg4(reinterpret_cast<const float *>(a.scratch + 2 * e)));
        } else {
            const float *s = reinterpret_cast<const float *>(a.scratch + 4 * e);
            u32x4 o[P];
            split8<P>(ldg4(s), ldg4(s + 4), o);
#pragma unroll
            for (int pl = 0; pl < P; ++pl) *reinterpret_cast<u32x4 *>(dst + pl * a.plb) = o[pl];
        }
    }
    zero_halo<P, R>(v, a.plb);
}

template <int P, int R, int H, int NC>
MPCD_DEV void run_op(const FArgs &a, const FOp &op, int64_t cand0, int64_t row0)
{
    switch (op.kind) {
    case FK_SAME5: conv_op<P, R, H, NC, FK_SAME5>(a, op, cand0, row0); break;
    case FK_DOWN3: conv_op<P, R, H, NC, FK_DOWN3>(a, op, cand0, row0); break;
    case FK_UP4: conv_op<P, R, H, NC, FK_UP4>(a, op, cand0, row0); break;
    default: conv_op<P, R, H, NC, FK_PW1>(a, op, cand0, row0); break;
    }
}

template <int P, int R, int H>
__global__ __launch_bounds__(FT) void unet_fused_kernel(const FArgs a)
{
    extern __shared__ __attribute__((aligned(16))) char sm[];
    constexpr int RC = R / 2, NCB = R * H / 64;
    static_assert(NCB >= 2 && NCB % 2 == 0, "R * H / 64 column tiles per wave must be even");
    const int tid = threadIdx.x;
    const int64_t cand0 = (int64_t)blockIdx.x * RC, row0 = (int64_t)blockIdx.x * R;
    const int d = a.d;

    // ---- stage x (both branches of each candidate) as 8 zero-padded channels, with its zero halo
    {
        const FView &v = a.xv;
        const int win = v.L + v.hl + v.hr;
        for (int i = tid; i < R * win; i += FT) {
            const int r = i / win, pw = i - r * win, p = pw - v.hl;
            const int64_t cand = cand0 + (r < RC ? r : r - RC);
            float xv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (p >= 0 && p < v.L && cand < a.batch)
                for (int k = 0; k < d; ++k) xv[k] = a.x[((size_t)cand * v.L + p) * d + k];
            u32x4 o[P];
            split8<P>(f32x4{xv[0], xv[1], xv[2], xv[3]}, f32x4{xv[4], xv[5], xv[6], xv[7]}, o);
#pragma unroll
            for (int pl = 0; pl < P; ++pl)
                *reinterpret_cast<u32x4 *>(sm + v.off + pl * a.plb + r * v.rowB + p * v.cs) = o[pl];
        }
    }
    __syncthreads();

    for (int oi = 0; oi < a.n_ops; ++oi) {
        const FOp &op = a.ops[oi];
        if (op.kind == FK_RESTORE) {
            restore_op<P, R>(a, op, row0);
        } else {
            if (op.half) run_op<P, R, H, NCB / 2>(a, op, cand0, row0);
            else run_op<P, R, H, NCB>(a, op, cand0, row0);
            if (op.out.hl + op.out.hr > 0 && op.epi != FE_EPS) zero_halo<P, R>(op.out, a.plb);
        }
        __syncthreads();
    }

    // ---- the denoise update of this step (or the raw eps of both branches, MODE_EPS)
    const float *E = reinterpret_cast<const float *>(sm + a.e_off);
    const int flat = H * d, quads = flat / 4;
    const StepPlan sp = a.plan ? a.plan[a.s] : StepPlan{};
    for (int i = tid; i < RC * quads; i += FT) {
        const int c = i / quads, qd = i - c * quads;
        const int64_t cand = cand0 + c;
        if (cand >= a.batch) continue;
        const size_t off = (size_t)cand * flat + 4 * qd;
        const f32x4 ec = *reinterpret_cast<const f32x4 *>(E + c * flat + 4 * qd);
        const f32x4 eu = *reinterpret_cast<const f32x4 *>(E + (c + RC) * flat + 4 * qd);
        if (a.mode == MODE_EPS) {
            *reinterpret_cast<f32x4 *>(a.eps_c + off) = ec;
            *reinterpret_cast<f32x4 *>(a.eps_u + off) = eu;
            continue;
        }
        const f32x4 xv = ldg4(a.x + off);
        f32x4 z = {0.f, 0.f, 0.f, 0.f};
        if (a.mode == MODE_DDPM_CFG && (sp.flags & PLAN_NOISE))
            z = a.noise ? ldg4(a.noise + (size_t)(a.s + 1) * a.batch * flat + off)
                        : philox_normal4(a.seed, (uint64_t)(a.goff + cand), (uint32_t)(a.s + 1), (uint32_t)qd);
        const f32x4 o = denoise_update4(sp, a.mode, a.clamp_x0, a.wp1, a.wf, xv, ec, eu, z);
        *reinterpret_cast<f32x4 *>(a.x + off) = o;
        if (a.amq) {
            const size_t qi = (size_t)cand * quads + qd;
            a.amq[qi] = absmax_bits4(a.s == 0 ? 0u : a.amq[qi], xv, o);
        }
        if (a.chain) *reinterpret_cast<f32x4 *>(a.chain + (size_t)(a.s + 1) * a.batch * flat + off) = o;
        if (a.last && a.x_out != a.x) *reinterpret_cast<f32x4 *>(a.x_out + off) = o;
    }
}

// ---- host: the program (op list) and the LDS placement

int cs_of(int C)  // bytes per position: an odd number of 16-byte units (conflict-free ds_read_b128 quarters)
{
    int cs = 2 * C;
    if (cs % 16) cs = (cs + 15) / 16 * 16;
    if (((cs / 16) & 1) == 0) cs += 16;
    return cs;
}
int ilog2(int v)
{
    int s = 0;
    while ((1 << s) < v) ++s;
    return (1 << s) == v ? s : -1;
}

struct Cfg {
    int P, R, H;
};
// the instantiated configurations: LDS of R rows must fit one CU (host-checked)
constexpr Cfg kCfgs[] = {{1, 6, 64}, {1, 4, 64}, {3, 4, 32}, {1, 8, 32}, {3, 2, 64}};

template <int P, int R, int H>
hipError_t launch_cfg(const FArgs &fa, unsigned grid, size_t lds, hipStream_t st)
{
    constexpr auto kfn = &unet_fused_kernel<P, R, H>;
    if (hipError_t e = allow_max_lds<kfn>(); e != hipSuccess) return e;
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(FT), lds, st, fa);
    return hipGetLastError();
}

hipError_t launch_any(int P, int R, int H, const FArgs &fa, unsigned grid, size_t lds, hipStream_t st)
{
#define C_(p, r, h) \
    if (P == p && R == r && H == h) return launch_cfg<p, r, h>(fa, grid, lds, st);
    C_(1, 6, 64) C_(1, 4, 64) C_(3, 4, 32) C_(1, 8, 32) C_(3, 2, 64)
#undef C_
    return hipErrorInvalidValue;
}

}  // namespace

struct UnetFusedPlan {
    int P = 0, R = 0, H = 0, d = 0;
    size_t lds = 0;
    int plb = 0, e_off = 0, stat_off = 0;
    FView xv{};
    std::vector<FOp> ops;
    FOp *ops_dev = nullptr;
    int64_t skip_elems_per_row = 0;  // scratch elements per row (h1)
    ~UnetFusedPlan()
    {
        if (ops_dev) (void)hipFree(ops_dev);
    }
};

void unet_fused_free(UnetFusedPlan *p) { delete p; }

// Build the program for ConditionedTemporalUnet(base 32, dim_mults (1, 2, 4)); nullptr (and *why) when the
// net or the numerics are not covered (the layer-by-layer path runs it instead).
UnetFusedPlan *unet_fused_prepare(const mpcd_net_desc &d, const UnetWeights &W, int rows_per_wg, std::string *why)
{
    auto no = [&](const char *m) -> UnetFusedPlan * {
        if (why) *why = m;
        return nullptr;
    };
    if (!W.ready || W.planes == 0) return no("fused U-Net: needs the bf16 / f16 matrix-core numerics");
    if (!d.cfg_masked) return no("fused U-Net: the CFG net (ConditionedTemporalUnet) only");
    if (d.base_dim != 32 || d.n_mults != 3 || d.mults[0] != 1 || d.mults[1] != 2 || d.mults[2] != 4)
        return no("fused U-Net: base 32, dim_mults (1, 2, 4) only");
    if (d.state_dim < 1 || d.state_dim > 8) return no("fused U-Net: state_dim 1..8");
    const int P = W.planes, H = d.horizon, dd = d.state_dim;
    if ((H * dd) % 4) return no("fused U-Net: H*d must be a multiple of 4");
    if (W.n_layers != 35) return no("fused U-Net: unexpected layer count");
    int R = 0;
    for (const Cfg &c : kCfgs)
        if (c.P == P && c.H == H && (rows_per_wg <= 0 || rows_per_wg == c.R)) {
            R = c.R;
            break;
        }
    if (!R) return no("fused U-Net: no instantiation for this horizon / numerics / rows per workgroup");

    auto *pl = new UnetFusedPlan;
    pl->P = P;
    pl->R = R;
    pl->H = H;
    pl->d = dd;
    const int H1 = H / 2, H2 = H / 4;
    // per-plane regions: A and B hold any level tensor, Z the third tensor of a projection block, the
    // concatenated up-path inputs, the staged x and the fp32 eps
    int rowA = 0;
    for (auto lc : {std::pair<int, int>{H, 32}, {H1, 64}, {H2, 128}, {H1, 32}, {H2, 64}})
        rowA = std::max(rowA, (lc.first + 4) * cs_of(lc.second));
    int rowZ = std::max({rowA, (H2 + 4) * cs_of(256), (H1 + 4) * cs_of(128), (H + 7) * cs_of(8), H * dd * 4});
    rowA = (rowA + 15) / 16 * 16;
    rowZ = (rowZ + 15) / 16 * 16;
    const int offA = 0, offB = R * rowA, offZ = 2 * R * rowA;
    pl->plb = offZ + R * rowZ;
    pl->stat_off = P * pl->plb;
    pl->e_off = offZ;
    const size_t stat_bytes = sizeof(float) * ((size_t)(R * (H >= 16 ? H / 16 : 1) * kGroups * 4) + (size_t)R * kGroups * 2);
    pl->lds = (size_t)pl->stat_off + stat_bytes;
    if (pl->lds > 160 * 1024) {
        delete pl;
        return no("fused U-Net: LDS over 160 KiB");
    }
    auto view = [&](int region, int L, int C, int ctot = 0, int ch0 = 0, int hl = 2, int hr = 2) {
        FView v{};
        v.cs = cs_of(ctot ? ctot : C);
        v.rowB = (L + hl + hr) * v.cs;
        v.off = region + hl * v.cs + 2 * ch0;
        v.L = L;
        v.C = C;
        v.hl = hl;
        v.hr = hr;
        return v;
    };
    pl->xv = view(offZ, H, 8, 0, 0, 2, 5);
    int li = 0;
    bool ok = true;
    auto op_of = [&](const ConvLayer &L, int epi, const FView &in, const FView &out, const FView *res, int lin) {
        FOp o{};
        o.w = L.wmx;
        o.bias = L.bias;
        o.gnw = L.gn_w;
        o.gnb = L.gn_b;
        o.kind = L.kind;
        o.epi = epi;
        o.cond_off = L.cond_off;
        o.cinp = L.cinp8;
        o.cpt_sh = L.cinp8 >= 32 ? ilog2(L.cinp8 / 32) : -1;
        o.kc = L.kc;
        o.nt_sh = ilog2(L.coutp / 16);
        o.cout = L.cout;
        o.lin = lin;
        o.lout = L.kind == UCONV_DOWN3 ? lin / 2 : L.kind == UCONV_UP4 ? 2 * lin : lin;
        o.lsh = ilog2(L.kind == UCONV_UP4 ? lin : o.lout);
        const int nt = L.coutp / 16, wc = 8 / std::max(nt, 1);
        const int ct = L.kind == UCONV_UP4 ? 2 * (R * lin / 16) : R * o.lout / 16;
        const int nc = nt >= 1 && nt <= 8 && ct % wc == 0 ? ct / wc : -1;
        const int ncb = R * H / 64;
        o.half = nc == ncb / 2 ? 1 : 0;
        if (nc != ncb && nc != ncb / 2) ok = false;
        if (L.kind == UCONV_UP4 && (R * lin / 16) % std::max(nc, 1)) ok = false;  // a wave's tiles in one parity
        if (o.cpt_sh < -1 || (L.cinp8 < 32 && L.cinp8 != 8) || o.nt_sh < 0 || o.lsh < 0) ok = false;
        if (L.cinp8 == 8 && in.hr < (L.kind == UCONV_SAME5 ? 5 : 3)) ok = false;  // tap slots past the kernel read the halo
        const bool gn = epi == FE_GN || epi == FE_GN_COND || epi == FE_GN_RES;
        if (gn) {
            o.cpg_sh = ilog2(L.cout / std::max(L.groups, 1));
            if (L.groups != kGroups || o.cpg_sh < 2 || o.cpg_sh > 4 || !L.gn_w || !L.gn_b || o.lout < 8) ok = false;
            if (epi == FE_GN_COND && L.cond_off < 0) ok = false;
        }
        o.in = in;
        o.out = out;
        if (res) o.res = *res;
        return o;
    };
    auto region_of = [&](const FView &v) { return v.off < offB ? 0 : v.off < offZ ? 1 : 2; };
    auto add = [&](int epi, const FView &in, const FView &out, const FView *res, int lin, int layer) {
        FOp o = op_of(W.layers[layer], epi, in, out, res, lin);
        o.alias_in = region_of(in) == region_of(out) ? 1 : 0;
        pl->ops.push_back(o);
        return (int)pl->ops.size() - 1;
    };
    // ResidualTemporalBlock (layers.py:323-355): [res 1x1] conv1 (GN Mish + cond) conv2 (GN Mish + res);
    // W.layers order per block: conv1, [res], conv2
    auto rtb = [&](const FView &in, const FView &h, const FView &out, const FView *res_tmp, int lin) {
        const int l1 = li, has_res = W.layers[li].cin != W.layers[li].cout;
        const int lr = li + 1, l2 = li + (has_res ? 2 : 1);
        li += has_res ? 3 : 2;
        const FView *res = &in;
        if (has_res) {
            add(FE_BIAS, in, *res_tmp, nullptr, lin, lr);
            res = res_tmp;
        }
        add(FE_GN_COND, in, h, nullptr, lin, l1);
        return add(FE_GN_RES, h, out, res, lin, l2);
    };
    const FView x = pl->xv;
    // level 0 (H positions, 32 channels)
    FView A0 = view(offA, H, 32), B0 = view(offB, H, 32);
    rtb(x, B0, A0, &A0, H);
    rtb(A0, B0, A0, nullptr, H);
    FView B0d = view(offB, H1, 32);
    add(FE_BIAS, A0, B0d, nullptr, H, li++);  // Downsample1d
    // level 1 (H/2, 64)
    FView A1 = view(offA, H1, 64), Z1 = view(offZ, H1, 64);
    rtb(B0d, Z1, A1, &A1, H1);
    const int h1op = rtb(A1, Z1, A1, nullptr, H1);
    pl->ops[h1op].spill = 1;  // h1 goes to the scratch (restored for the ups)
    pl->skip_elems_per_row = (int64_t)H1 * 64;
    FView B1d = view(offB, H2, 64);
    add(FE_BIAS, A1, B1d, nullptr, H1, li++);
    // level 2 (H/4, 128); h2 lands in the upper half of the 256-channel concat view
    FView A2 = view(offA, H2, 128), B2 = view(offB, H2, 128), Z2 = view(offZ, H2, 128);
    FView cat2hi = view(offZ, H2, 128, 256, 128), cat2lo = view(offZ, H2, 128, 256, 0), cat2 = view(offZ, H2, 256);
    rtb(B1d, Z2, A2, &A2, H2);
    rtb(A2, B2, cat2hi, nullptr, H2);
    // mid
    rtb(cat2hi, A2, B2, nullptr, H2);
    rtb(B2, A2, cat2lo, nullptr, H2);
    // ups.0: cat(mid, h2) -> 64
    FView A2u = view(offA, H2, 64), B2u = view(offB, H2, 64);
    rtb(cat2, B2u, A2u, &A2u, H2);
    rtb(A2u, B2u, A2u, nullptr, H2);
    FView cat1hi = view(offZ, H1, 64, 128, 64), cat1lo = view(offZ, H1, 64, 128, 0), cat1 = view(offZ, H1, 128);
    {
        FOp r{};
        r.kind = FK_RESTORE;
        r.spill = 1;
        r.out = cat1hi;
        pl->ops.push_back(r);
    }
    add(FE_BIAS, A2u, cat1lo, nullptr, H2, li++);  // Upsample1d -> lower half of the concat
    // ups.1: cat(up, h1) -> 32
    FView A1u = view(offA, H1, 32), B1u = view(offB, H1, 32);
    rtb(cat1, B1u, A1u, &A1u, H1);
    rtb(A1u, B1u, A1u, nullptr, H1);
    FView B0u = view(offB, H, 32), A0f = view(offA, H, 32);
    add(FE_BIAS, A1u, B0u, nullptr, H1, li++);
    // final Conv1dBlock + 1x1 conv -> eps (fp32, region Z plane 0)
    add(FE_GN, B0u, A0f, nullptr, H, li++);
    FView ev{};
    ev.off = offZ;
    add(FE_EPS, A0f, ev, nullptr, H, li++);
    if (!ok || li != W.n_layers) {
        delete pl;
        return no("fused U-Net: the program does not match the net");
    }
    if (hipMalloc(&pl->ops_dev, sizeof(FOp) * pl->ops.size()) != hipSuccess ||
        hipMemcpy(pl->ops_dev, pl->ops.data(), sizeof(FOp) * pl->ops.size(), hipMemcpyHostToDevice) != hipSuccess) {
        delete pl;
        return no("fused U-Net: op table upload");
    }
    return pl;
}

size_t unet_fused_scratch_bytes(const UnetFusedPlan &pl, int64_t batch)
{
    const int64_t wgs = (batch + pl.R / 2 - 1) / (pl.R / 2);
    return (size_t)wgs * pl.R * pl.skip_elems_per_row * (pl.P == 1 ? 2 : 4);
}

int unet_fused_rows_per_wg(const UnetFusedPlan &pl) { return pl.R; }

hipError_t unet_fused_step(const UnetFusedPlan &pl, const UnetFusedStep &s, hipStream_t st)
{
    FArgs fa{};
    fa.ops = pl.ops_dev;
    fa.n_ops = (int)pl.ops.size();
    fa.plb = pl.plb;
    fa.e_off = pl.e_off;
    fa.stat_off = pl.stat_off;
    fa.xv = pl.xv;
    fa.x = s.x;
    fa.batch = s.batch;
    fa.goff = s.goff;
    fa.d = pl.d;
    fa.mode = s.mode;
    fa.clamp_x0 = s.clamp_x0;
    fa.s = s.step;
    fa.last = s.last;
    fa.tp = s.tp;
    fa.cp = s.cp;
    fa.cp_stride = s.cp_stride;
    fa.plan = s.plan;
    fa.wp1 = s.wp1;
    fa.wf = s.wf;
    fa.noise = s.noise;
    fa.seed = s.seed;
    fa.chain = s.chain;
    fa.x_out = s.x_out;
    fa.amq = s.amq;
    fa.eps_c = s.eps_c;
    fa.eps_u = s.eps_u;
    fa.scratch = static_cast<char *>(s.scratch);
    const int64_t grid = (s.batch + pl.R / 2 - 1) / (pl.R / 2);
    if (grid <= 0 || grid > 0x7fffffff) return hipErrorInvalidValue;
    return launch_any(pl.P, pl.R, pl.H, fa, (unsigned)grid, pl.lds, st);
}
