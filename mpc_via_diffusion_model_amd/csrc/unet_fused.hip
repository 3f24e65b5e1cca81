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
#include <type_traits>
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

// device code reads the op table through the constant address space: every field is a scalar load of a
// provably uniform value (through a generic pointer the compiler cannot rule out aliasing stores, keeps the
// fields in VGPRs and wraps each buffer load whose descriptor comes from them in a waterfall loop)
typedef const FOp __attribute__((address_space(4))) COp;

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
    uint64_t *prof;           // diagnostics (MPCD_FUSED_PROF) or null: per workgroup < kProfWgs and op, wave 0's
                              // s_memtime at op start / GEMM done / statistics done / op done
};

// cross-lane sums on DPP (no LDS traffic): over an aligned group of 8 or 16 lanes inside one row of 16
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: every lane of the group gets the total)
MPCD_DEV float dpp_add(float v, int ctrl_sel)
{
    int o;
    switch (ctrl_sel) {
    case 0: o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false); break;
    case 1: o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false); break;
    case 2: o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false); break;
    default: o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false); break;
    }
    return v + __builtin_bit_cast(float, o);
}
MPCD_DEV float seg_sum(float v, int seg_len)
{
    v = dpp_add(v, 0);
    v = dpp_add(v, 1);
    v = dpp_add(v, 2);
    return seg_len == 16 ? dpp_add(v, 3) : v;
}
// rows 1 and 3 += the last lane of rows 0 and 2 (row_bcast:15): rows 1 / 3 hold the pair totals
MPCD_DEV float rows_pair_sum(float v)
{
    return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false));
}
// row 3 += lane 31 (rows 0 + 1, after rows_pair_sum; row_bcast:31): row 3 holds all four rows' total
MPCD_DEV float rows_quad_sum(float v)
{
    return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x143, 0x8, 0xF, false));
}

constexpr int kProfWgs = 64;
MPCD_DEV void prof_mark(const FArgs &a, int oi, int k)
{
    if (a.prof && blockIdx.x < (unsigned)kProfWgs && threadIdx.x == 0)  // one lane's vector store
        a.prof[((size_t)blockIdx.x * a.n_ops + oi) * 4 + k] = __builtin_amdgcn_s_memtime();
}

constexpr int kGroups = 8;  // GroupNorm groups of every 32 / 64 / 128-channel conv (group_norm_n_groups)

template <int R, int H>
constexpr int part_floats() { return R * (H >= 16 ? H / 16 : 1) * kGroups * 4; }

template <int P> constexpr int kDA = P == 1 ? 4 : 2;  // A (weight) chunks in flight: L2 latency
constexpr int kDB = 2;                                  // B (LDS) chunks in flight
template <int P> struct APre {                          // the next conv's first A chunks, loaded ahead
    u32x4 A[kDA<P>][P];
    bool valid = false;
};

// the op's column tile geometry for this wave: n-tile, first column tile, parity (UP4)
template <int R, int NC, int KIND>
MPCD_DEV void wave_tiles(COp &op, int wave, int &nt, int &t0, int &par)
{
    const int nt_sh = op.nt_sh;
    nt = wave & ((1 << nt_sh) - 1);
    t0 = (wave >> nt_sh) * NC;
    par = 0;
    if (KIND == FK_UP4) par = t0 >= ((R * op.lin) >> 4) ? 1 : 0;  // tiles per parity = R * lin / 16 (host: NC divides it)
}

// column of tile t0 + cc for this lane -> (row, output position, tap-0 input position)
template <int R, int KIND>
MPCD_DEV void col_map(COp &op, int t0, int cc, int col, int par, int &r, int &o, int &pos0)
{
    int c = (t0 + cc) * 16 + col;
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
}

template <int P>
MPCD_DEV __amdgpu_buffer_rsrc_t weight_rsrc(COp &op)
{
    const int npar = op.kind == FK_UP4 ? 2 : 1;
    return __builtin_amdgcn_make_buffer_rsrc((void *)op.w, (short)0, (int)((npar << op.nt_sh) * op.kc * P * 1024),
                                             0x00020000);
}
template <int P>
MPCD_DEV void load_a(const __amdgpu_buffer_rsrc_t &rs, COp &op, int par, int nt, int kc, int lane, u32x4 (&A)[P])
{
#pragma unroll
    for (int pl = 0; pl < P; ++pl) {
        const int soff = __builtin_amdgcn_readfirstlane((((((par << op.nt_sh) + nt) * op.kc) + kc) * P + pl) * 1024);
        A[pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, soff, 0));
    }
}

// issue the first A chunks of op `nop` (the next conv) for this wave, to land while this op's epilogue runs
template <int P, int R, int NCB>
MPCD_DEV void prefetch_next(COp &nop, int wave, int lane, APre<P> &pre)
{
    pre.valid = false;
    if (nop.kind == FK_RESTORE) return;
    const int NC = nop.half ? NCB / 2 : NCB;
    const int nt = wave & ((1 << nop.nt_sh) - 1), t0 = (wave >> nop.nt_sh) * NC;
    const int par = nop.kind == FK_UP4 && t0 >= ((R * nop.lin) >> 4) ? 1 : 0;
    const __amdgpu_buffer_rsrc_t rs = weight_rsrc<P>(nop);
#pragma unroll
    for (int s = 0; s < kDA<P>; ++s) load_a<P>(rs, nop, par, nt, min(s, nop.kc - 1), lane, pre.A[s]);
    pre.valid = true;
}

// ---- one conv of the program: GEMM + statistics + epilogue, NC 16-column tiles per wave
template <int P, int R, int H, int NC, int KIND>
MPCD_DEV void conv_op(const FArgs &a, COp &op, COp *nop, int64_t cand0, int64_t row0, int oi, APre<P> &pre)
{
    extern __shared__ __attribute__((aligned(16))) char sm[];
    constexpr int NCB = R * H / 64, DA = kDA<P>, DB = kDB;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 15, q = lane >> 4;
    const int plb = a.plb;
    int nt, t0, par;
    wave_tiles<R, NC, KIND>(op, wave, nt, t0, par);
    const int n0 = nt * 16 + 4 * q;
    const int epi = op.epi;
    const bool gn = epi == FE_GN || epi == FE_GN_COND || epi == FE_GN_RES;

    // ---- this op's per-channel parameters, loaded now so they land during the GEMM (the parameter blob
    // is only 4-byte aligned: scalar loads for bias / GroupNorm affine)
    f32x4 bias = {0.f, 0.f, 0.f, 0.f}, gw = bias, gb = bias, cv0 = bias, cv1 = bias;
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[e] = n0 + e < op.cout ? op.bias[n0 + e] : 0.f;
    if (gn) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            gw[e] = op.gnw[n0 + e];
            gb[e] = op.gnb[n0 + e];
        }
        if (epi == FE_GN_COND) {
            cv1 = ldg4(a.tp + op.cond_off + n0);  // masked branch: Linear(Mish(cat(t_emb, 0))) = the time part
            cv0 = (a.cp && !a.cp_stride) ? cv1 + ldg4(a.cp + op.cond_off + n0) : cv1;
        }
    }

    // ---- columns of the wave's tiles
    int bb[NC], cr[NC], co[NC];
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) {
        int pos0;
        col_map<R, KIND>(op, t0, cc, col, par, cr[cc], co[cc], pos0);
        bb[cc] = op.in.off + cr[cc] * op.in.rowB + pos0 * op.in.cs;
    }

    // ---- implicit GEMM: acc[cc] = channels nt*16 + 4q + e of column tile t0 + cc (bias added after)
    const int KC = op.kc;
    f32x4 acc[NC];
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) acc[cc] = f32x4{0.f, 0.f, 0.f, 0.f};
    const __amdgpu_buffer_rsrc_t rs = weight_rsrc<P>(op);
    // K walk, branch-free: cinp >= 32: tap = kc >> cpt_sh, channels ((kc mod 2^cpt_sh) * 32 + 8q); cinp = 8:
    // one chunk = 4 taps, lane quarter q takes tap 4kc + q, channels 0..7
    const int ics = op.in.cs, c8 = op.cpt_sh < 0 ? 1 : 0;
    const int tap_sh = c8 ? 0 : op.cpt_sh + 2, ci_mask = c8 ? 0 : (1 << op.cpt_sh) - 1;
    const int tap_q = c8 ? q : 0, ci_q = c8 ? 0 : 16 * q;
    auto koff = [&](int kc) -> int {
        const int tap = ((kc << 2) + tap_q) >> tap_sh;
        return (KIND == FK_UP4 ? -tap : tap) * ics + ((kc & ci_mask) << 6) + ci_q;
    };
    auto load_b = [&](u32x4 (&B)[NC][P], int kc) {
        const int ko = koff(min(kc, KC - 1));
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
    u32x4 A[DA][P];
    if (pre.valid) {
#pragma unroll
        for (int s = 0; s < DA; ++s)
#pragma unroll
            for (int pl = 0; pl < P; ++pl) A[s][pl] = pre.A[s][pl];
    } else {
#pragma unroll
        for (int s = 0; s < DA; ++s) load_a<P>(rs, op, par, nt, min(s, KC - 1), lane, A[s]);
    }
    pre.valid = false;
    u32x4 B[DB][NC][P];
#pragma unroll
    for (int s = 0; s < DB; ++s) load_b(B[s], s);
    constexpr int U = DA > DB ? DA : DB;  // DA and DB are powers of two: ring slots are compile-time
    auto step = [&](int k, int s) {       // chunk k = (multiple of U) + s
        mmas(A[s % DA], B[s % DB]);
        load_b(B[s % DB], k + DB);
        load_a<P>(rs, op, par, nt, min(k + DA, KC - 1), lane, A[s % DA]);
    };
    int kc = 0;
    for (; kc + U <= KC; kc += U) {
#pragma unroll
        for (int s = 0; s < U; ++s) step(kc + s, s);
    }
#pragma unroll
    for (int s = 0; s < U - 1; ++s)  // tail (its ring refills are clamped to the last chunk)
        if (kc + s < KC) step(kc + s, s);
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) acc[cc] = acc[cc] + bias;

    prof_mark(a, oi, 1);
    // ---- GroupNorm statistics from the accumulators
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
            // the segment's columns (8 or 16 lanes of one DPP row), then the group's lane quarters (rows)
            s1 = seg_sum(s1, seg_len);
            s2 = seg_sum(s2, seg_len);
            if (seg_len == 16) {  // every lane of a row holds its row total: row_bcast chains (writer: last row)
                if (qmask >= 1) {
                    s1 = rows_pair_sum(s1);
                    s2 = rows_pair_sum(s2);
                }
                if (qmask >= 3) {
                    s1 = rows_quad_sum(s1);
                    s2 = rows_quad_sum(s2);
                }
            } else {  // two 8-lane segments per row: symmetric exchanges across rows (every row gets the total)
                if (qmask >= 1) {
                    s1 += __shfl_xor(s1, 16);
                    s2 += __shfl_xor(s2, 16);
                }
                if (qmask >= 3) {
                    s1 += __shfl_xor(s1, 32);
                    s2 += __shfl_xor(s2, 32);
                }
            }
            if ((col & (seg_len - 1)) == 0 && (q & qmask) == qmask) {
                const int seg = ((t0 + cc) * 16 + col) >> seg_sh;
                *reinterpret_cast<f32x4 *>(part + (seg * kGroups + g) * 4) = f32x4{s1, s2, sh, 0.f};
            }
        }
        lds_barrier();
        if (tid < R * kGroups) {  // one (row, group) per thread: its equal-sized segments, fixed order
            using acc_t = typename std::conditional<P == 1, float, double>::type;
            const int r = tid / kGroups, gg = tid - r * kGroups;
            const int nseg = L >> seg_sh;  // 1, 2 or 4
            const acc_t n1 = (acc_t)(seg_len << op.cpg_sh), inv_n1 = (acc_t)1 / n1;  // powers of two: exact
            acc_t mk[4] = {0, 0, 0, 0}, m2 = 0, msum = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k < nseg) {
                    const f32x4 p = *reinterpret_cast<const f32x4 *>(part + ((r * nseg + k) * kGroups + gg) * 4);
                    mk[k] = (acc_t)p[2] + (acc_t)p[0] * inv_n1;
                    m2 += (acc_t)p[1] - (acc_t)p[0] * (acc_t)p[0] * inv_n1;
                    msum += mk[k];
                }
            }
            const acc_t mean = msum * ((acc_t)1 / (acc_t)nseg);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < nseg) m2 += n1 * (mk[k] - mean) * (mk[k] - mean);
            const acc_t var = m2 * (inv_n1 * ((acc_t)1 / (acc_t)nseg));
            stat[2 * tid] = (float)mean;
            stat[2 * tid + 1] = (float)((acc_t)1 / sqrt((var > 0 ? var : (acc_t)0) + (acc_t)1e-5));
        }
        lds_barrier();
    } else if (op.alias_in) {
        lds_barrier();
    }
    if (nop) prefetch_next<P, R, NCB>(*nop, wave, lane, pre);  // lands while this epilogue runs

    prof_mark(a, oi, 2);
    // ---- epilogue: GroupNorm affine -> Mish -> + cond / + residual, written as the next conv's planes
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
        if (op.spill) {  // the skip tensor, as the LDS holds it (fp16), or its fp32 value (re-split on restore);
                         // restore_op reads it back in this same lane (program order: no cross-wave hand-off)
            const size_t e = ((size_t)(row0 + r) * op.out.L + o) * op.out.C + n0;
            if constexpr (P == 1)
                *reinterpret_cast<u32x2 *>(a.scratch + 2 * e) = pk[0];
            else
                *reinterpret_cast<f32x4 *>(a.scratch + 4 * e) = v;
        }
    }
}

// zero halo positions of a view (every row, every plane, the view's channels)
template <int P, int R, typename View>
MPCD_DEV void zero_halo(const View &v, int plb)
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

// skip tensor back from the scratch into its LDS view: the RESTORE op carries the spilling conv's tile
// geometry (n-tiles, column tiles per wave, length), so every lane reads back exactly the elements it stored
template <int P, int R, int H, int NC>
MPCD_DEV void restore_op(const FArgs &a, COp &op, int64_t row0)
{
    extern __shared__ __attribute__((aligned(16))) char sm[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int col = lane & 15, q = lane >> 4;
    int nt, t0, par;
    wave_tiles<R, NC, FK_SAME5>(op, wave, nt, t0, par);
    const int n0 = nt * 16 + 4 * q;
    auto &v = op.out;
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) {
        int r, o, pos0;
        col_map<R, FK_SAME5>(op, t0, cc, col, 0, r, o, pos0);
        const size_t e = ((size_t)(row0 + r) * v.L + o) * v.C + n0;
        u32x2 pk[P];
        if constexpr (P == 1) {
            pk[0] = *reinterpret_cast<const u32x2 *>(a.scratch + 2 * e);
        } else {
            split4<P>(*reinterpret_cast<const f32x4 *>(a.scratch + 4 * e), pk);
        }
        char *dst = sm + v.off + r * v.rowB + o * v.cs + 2 * n0;
#pragma unroll
        for (int pl = 0; pl < P; ++pl) *reinterpret_cast<u32x2 *>(dst + pl * a.plb) = pk[pl];
    }
    zero_halo<P, R>(v, a.plb);
}

template <int P, int R, int H, int NC>
MPCD_DEV void run_op(const FArgs &a, COp &op, COp *nop, int64_t cand0, int64_t row0, int oi, APre<P> &pre)
{
    switch (op.kind) {
    case FK_SAME5: conv_op<P, R, H, NC, FK_SAME5>(a, op, nop, cand0, row0, oi, pre); break;
    case FK_DOWN3: conv_op<P, R, H, NC, FK_DOWN3>(a, op, nop, cand0, row0, oi, pre); break;
    case FK_UP4: conv_op<P, R, H, NC, FK_UP4>(a, op, nop, cand0, row0, oi, pre); break;
    case FK_PW1: conv_op<P, R, H, NC, FK_PW1>(a, op, nop, cand0, row0, oi, pre); break;
    default: restore_op<P, R, H, NC>(a, op, row0); break;
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
    APre<P> pre;
    // the first conv's weights are in flight while x is staged
    COp *ops = (COp *)(uintptr_t)a.ops;
    prefetch_next<P, R, NCB>(ops[0], __builtin_amdgcn_readfirstlane(tid >> 6), tid & 63, pre);

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
    lds_barrier();

    for (int oi = 0; oi < a.n_ops; ++oi) {
        COp &op = ops[oi];
        COp *nop = oi + 1 < a.n_ops ? &ops[oi + 1] : nullptr;
        prof_mark(a, oi, 0);
        if (op.half) run_op<P, R, H, NCB / 2>(a, op, nop, cand0, row0, oi, pre);
        else run_op<P, R, H, NCB>(a, op, nop, cand0, row0, oi, pre);
        if (op.kind != FK_RESTORE && op.out.hl + op.out.hr > 0 && op.epi != FE_EPS) zero_halo<P, R>(op.out, a.plb);
        lds_barrier();
        prof_mark(a, oi, 3);
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

// bytes per position of a C-channel plane: >= 2C and = 32 mod 64. A B-fragment read (ds_read_b128) has lane l
// read 16 bytes at column (l & 15) x cs + quarter (l >> 4) x 16; gfx950 services the wave in four lane groups
// ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, and the same + 32), and with cs = 32 mod 64 bytes every group's 16
// reads cover the 64 banks exactly once (an odd number of 16-byte units, the layer-by-layer kernels' rule, leaves
// two lanes of each group on the same banks: 2 LDS cycles per group instead of 1).
int cs_of(int C)
{
    int cs = (2 * C + 15) / 16 * 16;
    while (cs % 64 != 32) cs += 16;
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
    // activation views share their zero halos between rows: row r's positions L, L+1 are row r+1's -2, -1
    // (R * (L + 2) + 2 positions per view); the staged x keeps its own 2 + 5 (its tap-slot overrun reads must
    // never reach a neighbouring candidate's values)
    auto vbytes = [&](int L, int C) { return (R * (L + 2) + 2) * cs_of(C); };
    int regA = 0;
    for (auto lc : {std::pair<int, int>{H, 32}, {H1, 64}, {H2, 128}, {H1, 32}, {H2, 64}})
        regA = std::max(regA, vbytes(lc.first, lc.second));
    int regZ = std::max({regA, vbytes(H2, 256), vbytes(H1, 128), R * (H + 7) * cs_of(8), R * H * dd * 4});
    regA = (regA + 15) / 16 * 16;
    regZ = (regZ + 15) / 16 * 16;
    const int offA = 0, offB = regA, offZ = 2 * regA;
    pl->plb = offZ + regZ;
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
        v.rowB = (hr == 2 ? L + 2 : L + hl + hr) * v.cs;  // shared halos (hl = hr = 2), else per row
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
    {  // h1 back into the upper half of the 128-channel concat view, in the spilling conv's lane mapping
        FOp r = pl->ops[h1op];
        r.kind = FK_RESTORE;
        r.epi = FE_BIAS;
        r.spill = 1;
        r.alias_in = 0;
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
int unet_fused_n_ops(const UnetFusedPlan &pl) { return (int)pl.ops.size(); }
int unet_fused_prof_wgs() { return kProfWgs; }
void unet_fused_op_info(const UnetFusedPlan &pl, int i, int32_t out[6])
{
    const FOp &o = pl.ops[i];
    const int32_t v[6] = {o.kind, o.epi, o.cinp, o.cout, o.lout, o.kc};
    for (int k = 0; k < 6; ++k) out[k] = v[k];
}

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
    fa.prof = s.prof;
    const int64_t grid = (s.batch + pl.R / 2 - 1) / (pl.R / 2);
    if (grid <= 0 || grid > 0x7fffffff) return hipErrorInvalidValue;
    return launch_any(pl.P, pl.R, pl.H, fa, (unsigned)grid, pl.lds, st);
}
