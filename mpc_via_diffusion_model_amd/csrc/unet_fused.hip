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
// (the packed weights, unet_pack_mx) streams from L2 by buffer loads a few k-chunks ahead (the first chunks
// of the next conv are issued before this conv's epilogue). The only HBM traffic per step is x and the
// result, plus one skip tensor (h1) spilled to a scratch buffer while the lower levels run: it would not fit
// the LDS next to the others.
//
// The network is fixed, so the program (the 36 ops: convs + the h1 restore, their LDS views and tilings) is
// a compile-time table per (numerics P, rows R, horizon H): every shape, offset and branch of the device
// code is a constant; only the weight pointers come from a small runtime table (FPtr). Per conv: implicit
// GEMM on v_mfma_f32_16x16x32_{f16,bf16} - wave w owns NTW (1 or 2) consecutive n-tiles and NCW consecutive
// 16-column tiles of the R x L output columns (every wave has the same work; two n-tiles per wave read every
// B fragment once for two MFMAs: the LDS read rate is otherwise the MFMA rate); GroupNorm statistics straight
// from the accumulators (exact two-pass, DPP / permlane reductions inside the wave, or per-wave partials
// through LDS when a row spans two waves; fixed order: deterministic, independent of the batch and of the
// workgroup); the epilogue (bias, GroupNorm affine -> Mish -> + cond / + residual) in packed-fp32 registers,
// written as the next conv's planes.
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

constexpr int kNtwMax = 2;   // n-tiles per wave a conv may get: 1 preferred (2 everywhere measured slower, DESIGN.md
                             // §4), 2 where a 4-wave workgroup has more n-tiles than waves
constexpr int kGroups = 8;  // GroupNorm groups of every 32 / 64 / 128-channel conv (group_norm_n_groups)
constexpr int kWprMax = 8;  // waves a row of one conv's output may span (GroupNorm partials cross them through LDS)

enum { FK_SAME5 = 0, FK_DOWN3 = 1, FK_UP4 = 2, FK_PW1 = 3, FK_RESTORE = 4 };
enum { FE_BIAS = 0, FE_GN = 1, FE_GN_COND = 2, FE_GN_RES = 3, FE_EPS = 4 };
static_assert(FK_SAME5 == UCONV_SAME5 && FK_DOWN3 == UCONV_DOWN3 && FK_UP4 == UCONV_UP4 && FK_PW1 == UCONV_PW1,
              "conv kinds");

// ---- the program (compile time)

struct CView {
    int off, cs, rowB;  // byte offset in plane 0 of (row 0, position 0, first channel); bytes per position / row
    int L, C;           // positions, channels
};
struct COp {
    int kind, epi, layer;  // layer: index in UnetWeights::layers (the RESTORE op: the spilling conv's)
    int cinp, kc, nt_sh, cout, lin, lout;
    int ntw_sh, ncw;       // log2 n-tiles per wave; 16-column tiles per wave
    int cpg_sh;            // log2 channels per GroupNorm group
    int wpr;               // waves per row of the output (GroupNorm partial sums cross waves through LDS when > 1)
    int alias_in;          // the output overwrites the GEMM input region (barrier before the epilogue)
    int spill;             // also write the output to the skip scratch (RESTORE: read it back)
    CView in, res, out;
};
// MPCD_FUSED_GN1 = 1: GroupNorm statistics in one pass (sums and sums of squares reduced together,
// var = E[x^2] - mean^2) instead of the exact two-pass; experiment switch
#ifndef MPCD_FUSED_GN1
#define MPCD_FUSED_GN1 0
#endif
constexpr int kMaxOps = 40;
struct Prog {
    COp ops[kMaxOps];
    int n, plb, e_off, stat_off, lds, skip_elems_per_row, ok;
    CView xv;  // staged x: 8 channels, its own 2 + 5 zero positions per row
};

// bytes per position of a C-channel plane: >= 2C and = 32 mod 64. A B-fragment read (ds_read_b128) has lane l
// read 16 bytes at column (l & 15) x cs + quarter (l >> 4) x 16; gfx950 services the wave in four lane groups
// ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, and the same + 32), and with cs = 32 mod 64 bytes every group's 16
// reads cover the 64 banks exactly once (an odd number of 16-byte units leaves two lanes of each group on the
// same banks: 2 LDS cycles per group instead of 1).
constexpr int cs_of(int C)
{
    int cs = (2 * C + 15) / 16 * 16;
    while (cs % 64 != 32) cs += 16;
    return cs;
}
constexpr int ilog2c(int v)
{
    int s = 0;
    while ((1 << s) < v) ++s;
    return (1 << s) == v ? s : -1;
}

template <int P, int R, int H, int W>
constexpr Prog make_prog()
{
    Prog pg{};
    pg.ok = 1;
    const int H1 = H / 2, H2 = H / 4;
    // per-plane regions: A and B hold any level tensor, Z the third tensor of a projection block, the
    // concatenated up-path inputs, the staged x and the fp32 eps. Activation views share their zero halos
    // between rows (row r's positions L, L+1 are row r+1's -2, -1: R * (L + 2) + 2 positions per view).
    auto vbytes = [](int L, int C) { return (R * (L + 2) + 2) * cs_of(C); };
    int regA = 0;
    const int lc[5][2] = {{H, 32}, {H1, 64}, {H2, 128}, {H1, 32}, {H2, 64}};
    for (int i = 0; i < 5; ++i) regA = vbytes(lc[i][0], lc[i][1]) > regA ? vbytes(lc[i][0], lc[i][1]) : regA;
    int regZ = regA;
    const int zc[4] = {vbytes(H2, 256), vbytes(H1, 128), R * (H + 7) * cs_of(8), R * H * 8 * 4};
    for (int i = 0; i < 4; ++i) regZ = zc[i] > regZ ? zc[i] : regZ;
    regA = (regA + 15) / 16 * 16;
    regZ = (regZ + 15) / 16 * 16;
    const int offA = 0, offB = regA, offZ = 2 * regA;
    pg.plb = offZ + regZ;
    pg.e_off = offZ;
    pg.stat_off = P * pg.plb;
    pg.lds = pg.stat_off + 2 * 4 * R * kGroups * kWprMax;  // cross-wave GroupNorm partials [S1 | S2][row][group][part]
    auto view = [](int region, int L, int C, int ctot, int ch0) {
        CView v{};
        v.cs = cs_of(ctot ? ctot : C);
        v.rowB = (L + 2) * v.cs;
        v.off = region + 2 * v.cs + 2 * ch0;
        v.L = L;
        v.C = C;
        return v;
    };
    pg.xv.cs = cs_of(8);
    pg.xv.rowB = (H + 7) * pg.xv.cs;
    pg.xv.off = offZ + 2 * pg.xv.cs;
    pg.xv.L = H;
    pg.xv.C = 8;
    int li = 0;
    auto region_of = [&](const CView &v) { return v.off < offB ? 0 : v.off < offZ ? 1 : 2; };
    auto add = [&](int kind, int epi, int cin, int cout, const CView &in, const CView &out, const CView *res, int lin) {
        COp o{};
        o.kind = kind;
        o.epi = epi;
        o.layer = li++;
        o.cinp = cin <= 8 ? 8 : (cin + 31) / 32 * 32;
        const int ks = kind == FK_SAME5 ? 5 : kind == FK_DOWN3 ? 3 : kind == FK_UP4 ? 2 : 1;
        o.kc = (ks * o.cinp + 31) / 32;
        const int coutp = (cout + 15) / 16 * 16, nt = coutp / 16;
        o.nt_sh = ilog2c(nt);
        o.cout = cout;
        o.lin = lin;
        o.lout = kind == FK_DOWN3 ? lin / 2 : kind == FK_UP4 ? 2 * lin : lin;
        const int ct = kind == FK_UP4 ? 2 * (R * lin / 16) : R * o.lout / 16;  // column tiles
        const bool gn = epi == FE_GN || epi == FE_GN_COND || epi == FE_GN_RES;
        o.cpg_sh = gn ? ilog2c(cout / kGroups) : 0;
        if (gn && (o.cpg_sh < 2 || o.cpg_sh > 4 || o.lout < 8)) pg.ok = 0;
        // tiling: one n-tile per wave where the columns split evenly over the waves, else two; a wave's
        // columns in one UP4 parity, and (GroupNorm) whole rows or one half of a row
        o.ntw_sh = -1;
        for (int w = 0; w <= (nt >= 2 && kNtwMax >= 2 ? 1 : 0) && o.ntw_sh < 0; ++w) {
            const int ntg = nt >> w, wc = ntg >= 1 && ntg <= W ? W / ntg : 0;
            const int ncw = wc && ct % wc == 0 ? ct / wc : 0;
            if (ncw < 1 || (ncw << w) > 4 || (kind == FK_UP4 && (R * lin / 16) % ncw)) continue;
            const int wpr = gn && o.lout > 16 && (ncw * 16) % o.lout ? o.lout / (ncw * 16) : 1;
            if (wpr > kWprMax || (wpr > 1 && (o.lout != wpr * ncw * 16 || (wpr & (wpr - 1))))) continue;
            o.ntw_sh = w;
            o.ncw = ncw;
            o.wpr = wpr;
        }
        if (o.ntw_sh < 0 || o.nt_sh < 0) pg.ok = 0;
        o.in = in;
        o.out = out;
        if (res) o.res = *res;
        o.alias_in = region_of(in) == region_of(out) ? 1 : 0;
        if (pg.n >= kMaxOps) pg.ok = 0;
        else pg.ops[pg.n++] = o;
        return pg.n - 1;
    };
    // ResidualTemporalBlock (layers.py:323-355): [res 1x1] conv1 (GN Mish + cond) conv2 (GN Mish + res); the
    // layer table order per block is conv1, [res], conv2 (unet.hip unet_prepare)
    auto rtb = [&](int cin, int cout, const CView &in, const CView &h, const CView &out, const CView *res_tmp, int lin) {
        const int l1 = li;
        const bool has_res = cin != cout;
        const CView *res = &in;
        if (has_res) {
            li = l1 + 1;
            add(FK_PW1, FE_BIAS, cin, cout, in, *res_tmp, nullptr, lin);
            res = res_tmp;
        }
        li = l1;
        add(FK_SAME5, FE_GN_COND, cin, cout, in, h, nullptr, lin);
        li = l1 + (has_res ? 2 : 1);
        const int r = add(FK_SAME5, FE_GN_RES, cout, cout, h, out, res, lin);
        return r;
    };
    const CView x = pg.xv;
    const CView A0 = view(offA, H, 32, 0, 0), B0 = view(offB, H, 32, 0, 0);
    rtb(8, 32, x, B0, A0, &A0, H);  // cin = d <= 8 (zero-padded to 8 channels)
    rtb(32, 32, A0, B0, A0, nullptr, H);
    const CView B0d = view(offB, H1, 32, 0, 0);
    add(FK_DOWN3, FE_BIAS, 32, 32, A0, B0d, nullptr, H);  // Downsample1d
    const CView A1 = view(offA, H1, 64, 0, 0), Z1 = view(offZ, H1, 64, 0, 0);
    rtb(32, 64, B0d, Z1, A1, &A1, H1);
    const int h1op = rtb(64, 64, A1, Z1, A1, nullptr, H1);
    pg.ops[h1op].spill = 1;  // h1 goes to the scratch (restored for the ups)
    pg.skip_elems_per_row = H1 * 64;
    const CView B1d = view(offB, H2, 64, 0, 0);
    add(FK_DOWN3, FE_BIAS, 64, 64, A1, B1d, nullptr, H1);
    // level 2; h2 lands in the upper half of the 256-channel concat view
    const CView A2 = view(offA, H2, 128, 0, 0), B2 = view(offB, H2, 128, 0, 0), Z2 = view(offZ, H2, 128, 0, 0);
    const CView cat2hi = view(offZ, H2, 128, 256, 128), cat2lo = view(offZ, H2, 128, 256, 0), cat2 = view(offZ, H2, 256, 0, 0);
    rtb(64, 128, B1d, Z2, A2, &A2, H2);
    rtb(128, 128, A2, B2, cat2hi, nullptr, H2);
    rtb(128, 128, cat2hi, A2, B2, nullptr, H2);  // mid_block1
    rtb(128, 128, B2, A2, cat2lo, nullptr, H2);  // mid_block2
    // ups.0: cat(mid, h2) -> 64
    const CView A2u = view(offA, H2, 64, 0, 0), B2u = view(offB, H2, 64, 0, 0);
    rtb(256, 64, cat2, B2u, A2u, &A2u, H2);
    rtb(64, 64, A2u, B2u, A2u, nullptr, H2);
    const CView cat1hi = view(offZ, H1, 64, 128, 64), cat1lo = view(offZ, H1, 64, 128, 0), cat1 = view(offZ, H1, 128, 0, 0);
    {  // h1 back into the upper half of the 128-channel concat view, in the spilling conv's lane mapping
        COp r = pg.ops[h1op];
        r.kind = FK_RESTORE;
        r.epi = FE_BIAS;
        r.alias_in = 0;
        r.out = cat1hi;
        if (pg.n >= kMaxOps) pg.ok = 0;
        else pg.ops[pg.n++] = r;
    }
    add(FK_UP4, FE_BIAS, 64, 64, A2u, cat1lo, nullptr, H2);  // Upsample1d -> lower half of the concat
    // ups.1: cat(up, h1) -> 32
    const CView A1u = view(offA, H1, 32, 0, 0), B1u = view(offB, H1, 32, 0, 0);
    rtb(128, 32, cat1, B1u, A1u, &A1u, H1);
    rtb(32, 32, A1u, B1u, A1u, nullptr, H1);
    const CView B0u = view(offB, H, 32, 0, 0), A0f = view(offA, H, 32, 0, 0);
    add(FK_UP4, FE_BIAS, 32, 32, A1u, B0u, nullptr, H1);
    // final Conv1dBlock + 1x1 conv (cout = d, padded to one n-tile) -> eps (fp32, region Z plane 0)
    add(FK_SAME5, FE_GN, 32, 32, B0u, A0f, nullptr, H);
    CView ev{};
    ev.off = offZ;
    add(FK_PW1, FE_EPS, 32, 8, A0f, ev, nullptr, H);
    if (li != 35 || pg.lds > 160 * 1024) pg.ok = 0;
    return pg;
}

template <int P, int R, int H, int W>
struct ProgOf {
    static constexpr Prog v = make_prog<P, R, H, W>();
};

// ---- runtime tables and kernel arguments

struct FPtr {  // per op: weights (packed A fragments [parity][n-tile][k-chunk][plane][64][8]), bias, GroupNorm affine
    const uint16_t *w;
    const float *bias, *gnw, *gnb;
    int32_t cond_off;
    float inv;  // P = 2: 1 / the weights' power-of-two scale (the accumulator is unscaled before the bias)
};
typedef const FPtr __attribute__((address_space(4))) CPtr;  // scalar loads of provably uniform values

struct FArgs {
    const FPtr *ptrs;
    float *x;  // sampler state [B][H][d] (updated in place), or the input of MODE_EPS
    int64_t batch, goff;
    int32_t d, mode, clamp_x0, s, last, pad;
    const float *tp, *cp;  // tproj row of this step; cproj (per candidate or shared) or null
    int64_t cp_stride;
    const StepPlan *plan;
    float wp1, wf;
    const float *noise;
    uint64_t seed;
    float *chain, *x_out;
    uint32_t *amq;
    float *eps_c, *eps_u;  // MODE_EPS outputs
    char *scratch;         // skip spill: [row][L][C], fp16 (P = 1) or fp32 (P = 3)
    int64_t nblk;          // row blocks of R rows; workgroup b runs blocks b, b + gridDim.x, ... (persistent grid)
    uint64_t *prof;        // diagnostics (MPCD_FUSED_PROF) or null: per workgroup < kProfWgs and op, wave 0's
                           // s_memtime at op start / GEMM done / statistics done / op done
};

// ---- device helpers

// cross-lane sums on DPP (no LDS traffic): over an aligned group of 8 or 16 lanes inside one row of 16
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: every lane of the group gets the total)
template <int CTRL>
MPCD_DEV float dpp_add(float v)
{
    return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int SEG>
MPCD_DEV float seg_sum(float v)
{
    v = dpp_add<0xB1>(v);
    v = dpp_add<0x4E>(v);
    v = dpp_add<0x141>(v);
    if constexpr (SEG == 16) v = dpp_add<0x140>(v);
    return v;
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

// lane l + xor 16 / xor 32 partner sums on gfx950's permlane swaps (VALU, no LDS): with both operands the
// same register, the two results of v_permlane{16,32}_swap hold (own, partner) in complementary lanes, so
// their sum is v + v[l ^ 16] (v + v[l ^ 32]) in every lane
MPCD_DEV float xor16_sum(float v)
{
    const unsigned u = __builtin_bit_cast(unsigned, v);
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    const unsigned own = r[0], other = r[1];  // (bit_cast straight off r[1] reads r[0]: clang, ROCm 7.2)
    return __builtin_bit_cast(float, own) + __builtin_bit_cast(float, other);
}
MPCD_DEV float xor32_sum(float v)
{
    const unsigned u = __builtin_bit_cast(unsigned, v);
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    const unsigned own = r[0], other = r[1];  // (bit_cast straight off r[1] reads r[0]: clang, ROCm 7.2)
    return __builtin_bit_cast(float, own) + __builtin_bit_cast(float, other);
}
// sum over a (row segment, GroupNorm group): SEG columns (8 or 16 lanes of one DPP row) x the group's lane
// quarters (QMASK + 1 of them: 1, 2 or 4); every lane of the group gets the total. N independent sums step by
// step, so the DPP / permlane latencies of one chain hide behind the others.
template <int SEG, int QMASK, int N>
MPCD_DEV void group_sum_n(float (&v)[N])
{
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = dpp_add<0xB1>(v[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = dpp_add<0x4E>(v[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = dpp_add<0x141>(v[i]);
    if constexpr (SEG == 16) {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = dpp_add<0x140>(v[i]);
    }
    if constexpr (QMASK >= 1) {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = xor16_sum(v[i]);
    }
    if constexpr (QMASK >= 3) {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = xor32_sum(v[i]);
    }
}
template <int SEG, int QMASK>
MPCD_DEV float group_sum(float v)
{
    float a[1] = {v};
    group_sum_n<SEG, QMASK, 1>(a);
    return a[0];
}

// packed fp32 (v_pk_fma / v_pk_mul / v_pk_add: two lanes' worth per 4-cycle issue; the epilogue is VALU-bound)
MPCD_DEV f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
MPCD_DEV f32x2 lo2(const f32x4 &v) { return f32x2{v[0], v[1]}; }
MPCD_DEV f32x2 hi2(const f32x4 &v) { return f32x2{v[2], v[3]}; }
constexpr float kLog2e = 1.44269504088896341f, kLn2 = 0.693147180559945309f;
// Mish of a pair given in log2 units (z = y log2 e): y (1 - 2 / (n (n + 2) + 2)), n = e^y (common.h mish); four
// transcendentals, four packed ops
// The two transcendentals of a pair are issued together, followed by 2 wait states, so the packed op that reads
// them is never closer (packed reads of a v_exp / v_rcp result one wait state behind it gave wrong results on
// gfx950: profiles/r3_hazard_ab.txt; the compiler's scheduler alone kept that distance only by chance, and a new
// instantiation lost it). Same instructions as __builtin_amdgcn_exp2f / rcpf: the same bits.
MPCD_DEV f32x2 exp2_pair(f32x2 z)
{
    float a, b;
    asm("v_exp_f32 %0, %2\n\tv_exp_f32 %1, %3\n\ts_nop 1" : "=&v"(a), "=&v"(b) : "v"(z[0]), "v"(z[1]));
    return f32x2{a, b};
}
MPCD_DEV f32x2 rcp_pair(f32x2 x)
{
    float a, b;
    asm("v_rcp_f32 %0, %2\n\tv_rcp_f32 %1, %3\n\ts_nop 1" : "=&v"(a), "=&v"(b) : "v"(x[0]), "v"(x[1]));
    return f32x2{a, b};
}
MPCD_DEV f32x2 mish2_log2(f32x2 z)
{
    const f32x2 n = exp2_pair(z);
    const f32x2 den = fma2(n, n + 2.0f, f32x2{2.0f, 2.0f});
    const f32x2 r = rcp_pair(den);
    return z * fma2(r, f32x2{-2.0f * kLn2, -2.0f * kLn2}, f32x2{kLn2, kLn2});
}

// 1 / sqrt(x) for x >= 1e-5 (variance + eps): v_rsq_f32 and one Newton step (fp32-exact to ~1 ulp)
MPCD_DEV float rsqrt_nr(float x)
{
    const float r = __builtin_amdgcn_rsqf(x);
    return r * __builtin_fmaf(-0.5f * x * r, r, 1.5f);
}

constexpr int kProfWgs = 64;
MPCD_DEV void prof_mark(const FArgs &a, int n_ops, int oi, int k)
{
    if (a.prof && blockIdx.x < (unsigned)kProfWgs && threadIdx.x == 0)  // one lane's vector store
        a.prof[((size_t)blockIdx.x * n_ops + oi) * 4 + k] = __builtin_amdgcn_s_memtime();
}

template <int P> constexpr int kDA = P == 1 ? 4 : 2;  // A (weight) chunks in flight: L2 latency
constexpr int kDB = 2;                                  // B (LDS) chunks in flight
constexpr int kNTW = 2;                                 // n-tiles per wave, at most
template <int P> struct APre {                          // the next conv's first A chunks, loaded ahead
    u32x4 A[kDA<P>][kNTW][P];
};

template <int P, int R, int H, int W, int I>
struct OpGeo {  // the wave-independent constants of op I
    static constexpr COp op = ProgOf<P, R, H, W>::v.ops[I];
    static constexpr int NT = 1 << op.nt_sh, NTW = 1 << op.ntw_sh, NCW = op.ncw;
    static constexpr int ntg_sh = op.nt_sh - op.ntw_sh;                // log2 n-tile groups
    static constexpr int lcol = op.kind == FK_UP4 ? op.lin : op.lout;  // columns per row and parity
    static constexpr int lsh = ilog2c(lcol);
    static constexpr int tiles_par = R * op.lin / 16;                  // UP4: column tiles per parity
    static constexpr int npar = op.kind == FK_UP4 ? 2 : 1;
    static constexpr int wbytes = npar * NT * op.kc * P * 1024;        // packed weights of the op
};

template <int P>
MPCD_DEV __amdgpu_buffer_rsrc_t weight_rsrc(const uint16_t *w, int bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc((void *)w, (short)0, bytes, 0x00020000);
}
// k-chunk kc of n-tiles nt0 .. nt0 + NTW - 1 (every plane): one 16-byte buffer load per lane each
template <int P, int NT, int KC, int NTW>
MPCD_DEV void load_a(const __amdgpu_buffer_rsrc_t &rs, int par, int nt0, int kc, int lane, u32x4 (&A)[kNTW][P])
{
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int pl = 0; pl < P; ++pl) {
            const int soff = __builtin_amdgcn_readfirstlane(((((par * NT + nt0 + j) * KC) + kc) * P + pl) * 1024);
            A[j][pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, soff, 0));
        }
}

// this wave's first n-tile, first column tile and parity (UP4) in op I
template <int P, int R, int H, int W, int I>
MPCD_DEV void wave_tiles(int wave, int &nt0, int &t0, int &par)
{
    using G = OpGeo<P, R, H, W, I>;
    nt0 = (wave & ((1 << G::ntg_sh) - 1)) << G::op.ntw_sh;
    t0 = (wave >> G::ntg_sh) * G::NCW;
    par = G::op.kind == FK_UP4 && t0 >= G::tiles_par ? 1 : 0;  // make_prog: NCW divides tiles_par
}

// issue the first A chunks of op I for this wave (so they land while the previous op's epilogue runs)
template <int P, int R, int H, int W, int I>
MPCD_DEV void prefetch_op(const FArgs &a, int wave, int lane, APre<P> &pre)
{
    using G = OpGeo<P, R, H, W, I>;
    if constexpr (G::op.kind != FK_RESTORE) {
        CPtr &pp = reinterpret_cast<CPtr *>((uintptr_t)a.ptrs)[I];
        int nt0, t0, par;
        wave_tiles<P, R, H, W, I>(wave, nt0, t0, par);
        const __amdgpu_buffer_rsrc_t rs = weight_rsrc<P>(pp.w, G::wbytes);
#pragma unroll
        for (int s = 0; s < kDA<P>; ++s)
            load_a<P, G::NT, G::op.kc, G::NTW>(rs, par, nt0, s < G::op.kc ? s : G::op.kc - 1, lane, pre.A[s]);
    }
}

// zero the halo positions of a view (every plane, the view's channels): the R + 1 gaps of two positions each,
// in front of every row and after the last
template <int P, int R, int FT, int PLB, int OFF, int ROWB, int CS, int C>
MPCD_DEV void zero_halo()
{
    extern __shared__ __attribute__((aligned(16))) char sm[];
    constexpr int U = C / 8, N = P * (R + 1) * 2 * U;  // 16-byte units per position: C / 8
    for (int i = threadIdx.x; i < N; i += FT) {
        const int k = i % U, j = i / U, h = j & 1, rp = j >> 1;
        const int r = rp % (R + 1), pl = rp / (R + 1);
        *reinterpret_cast<u32x4 *>(sm + OFF + pl * PLB + r * ROWB + (h - 2) * CS + 16 * k) = u32x4{0u, 0u, 0u, 0u};
    }
}

// ---- one conv of the program: GEMM + statistics + epilogue
template <int P, int R, int H, int W, int I>
MPCD_DEV void conv_op(const FArgs &a, int64_t cand0, int64_t row0, int brn, APre<P> &pre)
{
    extern __shared__ __attribute__((aligned(16))) char sm[];
    using G = OpGeo<P, R, H, W, I>;
    constexpr COp op = G::op;
    constexpr int NCW = G::NCW, NTW = G::NTW, NT = G::NT, KC = op.kc, KIND = op.kind, EPI = op.epi;
    constexpr int DA = kDA<P>, DB = kDB;
    constexpr int PLB = ProgOf<P, R, H, W>::v.plb, N_OPS = ProgOf<P, R, H, W>::v.n;
    constexpr bool GN = EPI == FE_GN || EPI == FE_GN_COND || EPI == FE_GN_RES;
    static_assert(!(GN && op.alias_in), "GroupNorm ops write a region their GEMM does not read");
    static_assert(EPI != FE_EPS || NTW == 1, "the eps conv has one n-tile");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 15, q = lane >> 4;
    int nt0, t0, par;
    wave_tiles<P, R, H, W, I>(wave, nt0, t0, par);
    int n0[NTW];  // first of the lane's 4 output channels, per n-tile of the wave
#pragma unroll
    for (int j = 0; j < NTW; ++j) n0[j] = (nt0 + j) * 16 + 4 * q;
    CPtr &pp = reinterpret_cast<CPtr *>((uintptr_t)a.ptrs)[I];

    // ---- this op's per-channel parameters, loaded now so they land during the GEMM (the parameter blob is only
    // 4-byte aligned: scalar loads for bias / GroupNorm affine)
    // cond: cv1 = the masked branch's Linear(Mish(cat(t_emb, 0))) (the time part), cvs = the shared context
    // part (when the context is one row) - both loaded unconditionally (no branch, no wait before the GEMM)
    const bool shared_cp = a.cp && !a.cp_stride;
    f32x4 bias[NTW], gw[NTW], gb[NTW], cvs[NTW], cv1[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        bias[j] = gw[j] = gb[j] = cvs[j] = cv1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if constexpr (EPI == FE_EPS)
                bias[j][e] = n0[j] + e < a.d ? pp.bias[n0[j] + e] : 0.f;
            else
                bias[j][e] = pp.bias[n0[j] + e];
            if constexpr (GN) {
                gw[j][e] = pp.gnw[n0[j] + e];
                gb[j][e] = pp.gnb[n0[j] + e];
            }
        }
        if constexpr (EPI == FE_GN_COND) {
            cv1[j] = ldg4(a.tp + pp.cond_off + n0[j]);
            cvs[j] = ldg4((shared_cp ? a.cp : a.tp) + pp.cond_off + n0[j]);
        }
    }

    // ---- columns of the wave's tiles: (row, output position) and the tap-0 input position
    int bb[NCW], cr[NCW], co[NCW];
#pragma unroll
    for (int cc = 0; cc < NCW; ++cc) {
        int c = (t0 + cc) * 16 + col, pos0;
        if constexpr (KIND == FK_UP4) {
            c -= par * G::tiles_par * 16;
            cr[cc] = c >> G::lsh;
            const int m = c & (op.lin - 1);
            pos0 = par ? m + 1 : m;  // slot s reads position pos0 - s (ConvTranspose1d k4 s2 p1)
            co[cc] = 2 * m + par;
        } else {
            cr[cc] = c >> G::lsh;
            co[cc] = c & (op.lout - 1);
            pos0 = KIND == FK_SAME5 ? co[cc] - 2 : KIND == FK_DOWN3 ? 2 * co[cc] - 1 : co[cc];
        }
        bb[cc] = op.in.off + cr[cc] * op.in.rowB + pos0 * op.in.cs;
    }

    // ---- implicit GEMM: acc[j][cc] = channels (nt0 + j)*16 + 4q + e of column tile t0 + cc (bias added after)
    f32x4 acc[NTW][NCW];
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int cc = 0; cc < NCW; ++cc) acc[j][cc] = f32x4{0.f, 0.f, 0.f, 0.f};
    const __amdgpu_buffer_rsrc_t rs = weight_rsrc<P>(pp.w, G::wbytes);
    // K walk: cinp >= 32: chunk kc = tap kc >> log2(cinp/32), channels (kc mod (cinp/32)) * 32 + 8q; cinp = 8:
    // one chunk = 4 taps, lane quarter q takes tap 4kc + q, channels 0..7
    auto koff = [&](int kc) -> int {
        int tap, ci;
        if constexpr (op.cinp == 8) {
            tap = 4 * kc + q;
            ci = 0;
        } else {
            constexpr int cpt = op.cinp / 32;
            tap = kc / cpt;
            ci = (kc % cpt) * 32 + 8 * q;
        }
        return (KIND == FK_UP4 ? -tap : tap) * op.in.cs + 2 * ci;
    };
    auto load_b = [&](u32x4 (&B)[NCW][P], int kc) {
        const int ko = koff(kc < KC ? kc : KC - 1);
#pragma unroll
        for (int cc = 0; cc < NCW; ++cc)
#pragma unroll
            for (int pl = 0; pl < P; ++pl) B[cc][pl] = *reinterpret_cast<const u32x4 *>(sm + bb[cc] + ko + pl * PLB);
    };
    auto mmas = [&](const u32x4 (&A)[kNTW][P], const u32x4 (&B)[NCW][P]) {
#pragma unroll
        for (int i = 0; i < NPROD(P); ++i)
#pragma unroll
            for (int j = 0; j < NTW; ++j)
#pragma unroll
                for (int cc = 0; cc < NCW; ++cc) acc[j][cc] = mma<P>(A[j][PA<P>(i)], B[cc][PB<P>(i)], acc[j][cc]);
    };
    // the A ring: its first chunks were issued before the previous op's epilogue (P = 1: the prefetch registers
    // themselves; P = 3: a copy, which schedules the six-product K loop better)
    u32x4 Acopy[P == 1 ? 1 : DA][kNTW][P];
    u32x4(&A)[DA][kNTW][P] = *[&]() -> u32x4(*)[DA][kNTW][P] {
        if constexpr (P == 1) {
            return &pre.A;
        } else {
#pragma unroll
            for (int s = 0; s < DA; ++s)
#pragma unroll
                for (int j = 0; j < NTW; ++j)
#pragma unroll
                    for (int pl = 0; pl < P; ++pl) Acopy[s][j][pl] = pre.A[s][j][pl];
            return &Acopy;
        }
    }();
    u32x4 B[DB][NCW][P];
#pragma unroll
    for (int s = 0; s < DB; ++s) load_b(B[s], s);
    constexpr int U = DA > DB ? DA : DB;  // DA and DB are powers of two: ring slots are compile-time
    auto step = [&](int k, int s) {       // chunk k = (multiple of U) + s; refills clamped to the last chunk
        mmas(A[s % DA], B[s % DB]);
        load_b(B[s % DB], k + DB);
        const int kn = k + DA < KC ? k + DA : KC - 1;
        load_a<P, NT, KC, NTW>(rs, par, nt0, kn, lane, A[s % DA]);
        // keep the refills where they are: the scheduler would otherwise sink each load next to its use (to
        // shorten live ranges), leaving one chunk in flight and the L2 latency exposed at every MFMA
        __builtin_amdgcn_sched_barrier(0);
    };
    int kc = 0;
    for (; kc + U <= KC; kc += U) {
#pragma unroll
        for (int s = 0; s < U; ++s) step(kc + s, s);
    }
#pragma unroll
    for (int s = 0; s < U - 1; ++s)
        if (kc + s < KC) step(kc + s, s);
    if constexpr (P == 2) {  // unscale (exact: a power of two), then the bias
        const float inv = pp.inv;
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int cc = 0; cc < NCW; ++cc) acc[j][cc] = acc[j][cc] * inv + bias[j];
    } else {
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int cc = 0; cc < NCW; ++cc) acc[j][cc] = acc[j][cc] + bias[j];
    }

    if constexpr (I + 1 < N_OPS) prefetch_op<P, R, H, W, I + 1>(a, wave, lane, pre);  // lands during the epilogue
    prof_mark(a, N_OPS, I, 1);
    // ---- GroupNorm statistics per (row, group): a group's channels are 1, 2 or 4 lane quarters of one n-tile,
    // its columns the DPP-row lanes of the wave's tiles in that row. Exact two-pass (mean, then the centred sum of
    // squares); fixed order: the same bits for any batch, workgroup or tiling of the other ops.
    float mean[NTW][NCW], rstd[NTW][NCW];
    constexpr int QMASK = GN ? (1 << (op.cpg_sh - 2)) - 1 : 0;  // lane quarters per group - 1: 0, 1 or 3
    if constexpr (GN && op.wpr >= 2) {
        // a row spans WPR waves (the wave's NCW tiles are one part of it): per-wave partial sums through LDS, added in
        // wave order (the same order for every batch and workgroup); two barriers per op
        constexpr int WPR = op.wpr;
        constexpr float inv_n = 1.0f / (float)(op.lout << op.cpg_sh);
        float *st = reinterpret_cast<float *>(sm + ProgOf<P, R, H, W>::v.stat_off);  // [S1 | S2][row][group][part]
        constexpr int S2 = R * kGroups * kWprMax;
        const int row = cr[0], part = (t0 / NCW) & (WPR - 1);
        const bool leader = col == 0 && (q & QMASK) == 0;
        auto sum_parts = [&](const float *p) {
            float v = p[0];
#pragma unroll
            for (int i = 1; i < WPR; ++i) v = v + p[i];
            return v;
        };
        int slot[NTW];
        float m[NTW];
#if MPCD_FUSED_GN1
        // one pass, one barrier: both partial sums of each part of the row through LDS together
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            slot[j] = (row * kGroups + (n0[j] >> op.cpg_sh)) * kWprMax;
            f32x2 p1 = lo2(acc[j][0]) + hi2(acc[j][0]);
            f32x2 p2 = fma2(hi2(acc[j][0]), hi2(acc[j][0]), lo2(acc[j][0]) * lo2(acc[j][0]));
#pragma unroll
            for (int cc = 1; cc < NCW; ++cc) {
                const f32x2 a0 = lo2(acc[j][cc]), a1 = hi2(acc[j][cc]);
                p1 += a0 + a1;
                p2 = fma2(a1, a1, fma2(a0, a0, p2));
            }
            float ss[2] = {p1[0] + p1[1], p2[0] + p2[1]};
            group_sum_n<16, QMASK, 2>(ss);
            if (leader) {
                st[slot[j] + part] = ss[0];
                st[S2 + slot[j] + part] = ss[1];
            }
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            m[j] = sum_parts(st + slot[j]) * inv_n;
            const float rs = rsqrt_nr(fmaxf(sum_parts(st + S2 + slot[j]) * inv_n - m[j] * m[j], 0.f) + 1e-5f);
#pragma unroll
            for (int cc = 0; cc < NCW; ++cc) {
                mean[j][cc] = m[j];
                rstd[j][cc] = rs;
            }
        }
#else
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            slot[j] = (row * kGroups + (n0[j] >> op.cpg_sh)) * kWprMax;
            f32x2 p1 = lo2(acc[j][0]) + hi2(acc[j][0]);
#pragma unroll
            for (int cc = 1; cc < NCW; ++cc) p1 += lo2(acc[j][cc]) + hi2(acc[j][cc]);
            const float s1 = group_sum<16, QMASK>(p1[0] + p1[1]);
            if (leader) st[slot[j] + part] = s1;
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            m[j] = sum_parts(st + slot[j]) * inv_n;
            const f32x2 mm = {-m[j], -m[j]};
            f32x2 p2 = {0.f, 0.f};
#pragma unroll
            for (int cc = 0; cc < NCW; ++cc) {
                const f32x2 d0 = lo2(acc[j][cc]) + mm, d1 = hi2(acc[j][cc]) + mm;
                p2 = fma2(d1, d1, fma2(d0, d0, p2));
            }
            const float s2 = group_sum<16, QMASK>(p2[0] + p2[1]);
            if (leader) st[S2 + slot[j] + part] = s2;
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const float rs = rsqrt_nr(sum_parts(st + S2 + slot[j]) * inv_n + 1e-5f);
#pragma unroll
            for (int cc = 0; cc < NCW; ++cc) {
                mean[j][cc] = m[j];
                rstd[j][cc] = rs;
            }
        }
#endif
    } else if constexpr (GN) {  // every (row, group) inside the wave
        constexpr int L = op.lout, SEG = L < 16 ? L : 16, TPR = L > 16 ? L / 16 : 1;  // column tiles per row
        constexpr float inv_n = 1.0f / (float)(L << op.cpg_sh);
        static_assert(NCW % TPR == 0, "a wave's column tiles are whole rows");
        constexpr int NR = NCW / TPR, NS = NTW * NR;  // (n-tile, row) sums of the wave, reduced side by side
#if MPCD_FUSED_GN1
        // one pass: the sums and the sums of squares reduced side by side (one DPP chain's latency),
        // var = E[x^2] - mean^2 (clamped at 0)
        float ss[2 * NS];
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                f32x2 p1 = lo2(acc[j][r * TPR]) + hi2(acc[j][r * TPR]);
                f32x2 p2 = fma2(hi2(acc[j][r * TPR]), hi2(acc[j][r * TPR]), lo2(acc[j][r * TPR]) * lo2(acc[j][r * TPR]));
#pragma unroll
                for (int t = 1; t < TPR; ++t) {
                    const f32x2 a0 = lo2(acc[j][r * TPR + t]), a1 = hi2(acc[j][r * TPR + t]);
                    p1 += a0 + a1;
                    p2 = fma2(a1, a1, fma2(a0, a0, p2));
                }
                ss[j * NR + r] = p1[0] + p1[1];
                ss[NS + j * NR + r] = p2[0] + p2[1];
            }
        group_sum_n<SEG, QMASK, 2 * NS>(ss);
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float m = ss[j * NR + r] * inv_n;
                const float var = fmaxf(ss[NS + j * NR + r] * inv_n - m * m, 0.f);
                const float rs = rsqrt_nr(var + 1e-5f);
#pragma unroll
                for (int t = 0; t < TPR; ++t) {
                    mean[j][r * TPR + t] = m;
                    rstd[j][r * TPR + t] = rs;
                }
            }
#else
        float s1[NS], s2[NS];
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                f32x2 p1 = lo2(acc[j][r * TPR]) + hi2(acc[j][r * TPR]);
#pragma unroll
                for (int t = 1; t < TPR; ++t) p1 += lo2(acc[j][r * TPR + t]) + hi2(acc[j][r * TPR + t]);
                s1[j * NR + r] = p1[0] + p1[1];
            }
        group_sum_n<SEG, QMASK, NS>(s1);
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float m = s1[j * NR + r] * inv_n;
                const f32x2 mm = {-m, -m};
                f32x2 p2 = {0.f, 0.f};
#pragma unroll
                for (int t = 0; t < TPR; ++t) {
                    const f32x2 d0 = lo2(acc[j][r * TPR + t]) + mm, d1 = hi2(acc[j][r * TPR + t]) + mm;
                    p2 = fma2(d1, d1, fma2(d0, d0, p2));
                }
                s2[j * NR + r] = p2[0] + p2[1];
            }
        group_sum_n<SEG, QMASK, NS>(s2);
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float m = s1[j * NR + r] * inv_n, rs = rsqrt_nr(s2[j * NR + r] * inv_n + 1e-5f);
#pragma unroll
                for (int t = 0; t < TPR; ++t) {
                    mean[j][r * TPR + t] = m;
                    rstd[j][r * TPR + t] = rs;
                }
            }
#endif
    } else if constexpr (op.alias_in) {
        lds_barrier();
    }

    prof_mark(a, N_OPS, I, 2);
    // ---- epilogue: GroupNorm affine -> Mish -> + cond / + residual, written as the next conv's planes.
    // LDS reads of every tile first (residual), then the arithmetic, then the writes.
    f32x4 v[NTW][NCW];
    u32x2 rp[NTW][NCW][P];
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int cc = 0; cc < NCW; ++cc) {
            v[j][cc] = acc[j][cc];
            if constexpr (EPI == FE_GN_RES) {
                const char *s = sm + op.res.off + cr[cc] * op.res.rowB + co[cc] * op.res.cs + 2 * n0[j];
#pragma unroll
                for (int pl = 0; pl < P; ++pl) rp[j][cc][pl] = *reinterpret_cast<const u32x2 *>(s + pl * PLB);
            }
        }
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        // GroupNorm affine in log2 units: z = ((x - mean) rstd gamma + beta) log2 e
        const f32x2 gl0 = lo2(gw[j]) * kLog2e, gl1 = hi2(gw[j]) * kLog2e;
        const f32x2 bl0 = lo2(gb[j]) * kLog2e, bl1 = hi2(gb[j]) * kLog2e;
#pragma unroll
        for (int cc = 0; cc < NCW; ++cc) {
            if constexpr (GN) {
                const float r = rstd[j][cc], mr = -mean[j][cc] * r;
                const f32x2 rr = {r, r}, mm = {mr, mr};
                const f32x2 y0 = mish2_log2(fma2(fma2(lo2(v[j][cc]), rr, mm), gl0, bl0));
                const f32x2 y1 = mish2_log2(fma2(fma2(hi2(v[j][cc]), rr, mm), gl1, bl1));
                v[j][cc] = f32x4{y0[0], y0[1], y1[0], y1[1]};
            }
            if constexpr (EPI == FE_GN_COND) {
                // R = 1: the workgroup's one row is branch brn of candidate cand0; else rows [0, R/2) context
                const bool masked = R == 1 ? brn != 0 : cr[cc] >= R / 2;
                f32x4 cv = masked || !shared_cp ? cv1[j] : cv1[j] + cvs[j];
                if (!masked && a.cp && a.cp_stride) {
                    const int64_t cand = R == 1 ? cand0 : cand0 + cr[cc];
                    if (cand < a.batch) cv = cv + ldg4(a.cp + (size_t)cand * a.cp_stride + pp.cond_off + n0[j]);
                }
                v[j][cc] = v[j][cc] + cv;
            } else if constexpr (EPI == FE_GN_RES) {
                v[j][cc] = v[j][cc] + join4<P>(rp[j][cc]);
            }
        }
    }
    if constexpr (EPI == FE_EPS) {  // the net's output (cout = d): fp32 for the update
        float *E = reinterpret_cast<float *>(sm + ProgOf<P, R, H, W>::v.e_off);
#pragma unroll
        for (int cc = 0; cc < NCW; ++cc)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (n0[0] + e < a.d) E[(cr[cc] * H + co[cc]) * a.d + n0[0] + e] = v[0][cc][e];
    } else {
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int cc = 0; cc < NCW; ++cc) {
                u32x2 pk[P];
                split4<P>(v[j][cc], pk);
                char *dst = sm + op.out.off + cr[cc] * op.out.rowB + co[cc] * op.out.cs + 2 * n0[j];
#pragma unroll
                for (int pl = 0; pl < P; ++pl) *reinterpret_cast<u32x2 *>(dst + pl * PLB) = pk[pl];
                if constexpr (op.spill) {  // the skip tensor as the LDS holds it (fp16), or its fp32 value (re-split
                                           // on restore); restore_op reads it back in this same lane (program order)
                    const size_t e = ((size_t)(row0 + cr[cc]) * op.out.L + co[cc]) * op.out.C + n0[j];
                    if constexpr (P == 1)
                        *reinterpret_cast<u32x2 *>(a.scratch + 2 * e) = pk[0];
                    else
                        *reinterpret_cast<f32x4 *>(a.scratch + 4 * e) = v[j][cc];
                }
            }
        zero_halo<P, R, 64 * W, PLB, op.out.off, op.out.rowB, op.out.cs, op.out.C>();
    }
}

// skip tensor back from the scratch into its LDS view: the RESTORE op carries the spilling conv's tile
// geometry (n-tiles, column tiles per wave, length), so every lane reads back exactly the elements it stored
template <int P, int R, int H, int W, int I>
MPCD_DEV void restore_op(const FArgs &a, int64_t row0)
{
    extern __shared__ __attribute__((aligned(16))) char sm[];
    using G = OpGeo<P, R, H, W, I>;
    constexpr COp op = G::op;
    constexpr int PLB = ProgOf<P, R, H, W>::v.plb, NTW = G::NTW, NCW = G::NCW;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int col = lane & 15, q = lane >> 4;
    int nt0, t0, par;
    wave_tiles<P, R, H, W, I>(wave, nt0, t0, par);
    u32x2 pk[NTW][NCW][P];
    int cr[NCW], co[NCW];
#pragma unroll
    for (int cc = 0; cc < NCW; ++cc) {
        const int c = (t0 + cc) * 16 + col;
        cr[cc] = c >> G::lsh;
        co[cc] = c & (op.lout - 1);
    }
#pragma unroll
    for (int j = 0; j < NTW; ++j)  // every load in flight before the first LDS write
#pragma unroll
        for (int cc = 0; cc < NCW; ++cc) {
            const size_t e = ((size_t)(row0 + cr[cc]) * op.out.L + co[cc]) * op.out.C + (nt0 + j) * 16 + 4 * q;
            if constexpr (P == 1)
                pk[j][cc][0] = *reinterpret_cast<const u32x2 *>(a.scratch + 2 * e);
            else
                split4<P>(*reinterpret_cast<const f32x4 *>(a.scratch + 4 * e), pk[j][cc]);
        }
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int cc = 0; cc < NCW; ++cc) {
            char *dst = sm + op.out.off + cr[cc] * op.out.rowB + co[cc] * op.out.cs + 2 * ((nt0 + j) * 16 + 4 * q);
#pragma unroll
            for (int pl = 0; pl < P; ++pl) *reinterpret_cast<u32x2 *>(dst + pl * PLB) = pk[j][cc][pl];
        }
    zero_halo<P, R, 64 * W, PLB, op.out.off, op.out.rowB, op.out.cs, op.out.C>();
}

template <int P, int R, int H, int W, int I>
MPCD_DEV void run_ops(const FArgs &a, int64_t cand0, int64_t row0, int brn, APre<P> &pre)
{
    constexpr int N_OPS = ProgOf<P, R, H, W>::v.n;
    if constexpr (I < N_OPS) {
        prof_mark(a, N_OPS, I, 0);
        if constexpr (ProgOf<P, R, H, W>::v.ops[I].kind == FK_RESTORE) {
            restore_op<P, R, H, W, I>(a, row0);
            if constexpr (I + 1 < N_OPS) prefetch_op<P, R, H, W, I + 1>(a, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                                                                     threadIdx.x & 63, pre);
        } else {
            conv_op<P, R, H, W, I>(a, cand0, row0, brn, pre);
        }
        lds_barrier();
        prof_mark(a, N_OPS, I, 3);
        run_ops<P, R, H, W, I + 1>(a, cand0, row0, brn, pre);
    }
}

template <int P, int R, int H, int W, bool PERS>
__global__ __launch_bounds__(64 * W) void unet_fused_kernel(const FArgs a)
{
    constexpr int FT = 64 * W;
    extern __shared__ __attribute__((aligned(16))) char sm[];
    constexpr Prog pg = ProgOf<P, R, H, W>::v;
    static_assert(pg.ok, "fused U-Net program does not fit this (P, R, H)");
    constexpr int RC = R / 2, PLB = pg.plb;
    const int tid = threadIdx.x;
    const int d = a.d;
    APre<P> pre;
    // Row blocks blockIdx.x, + gridDim.x, ...: a grid of one block per row block runs one iteration; a persistent
    // grid (MPCD_FUSED_PERSIST) keeps each CU's workgroups walking the net together, block after block, so the
    // weights of the ops in flight stay in the XCD's L2 instead of every late-starting workgroup re-fetching them.
    for (int64_t blk = blockIdx.x; blk < a.nblk; blk += gridDim.x) {
    // R = 1 (the fp32-accurate H = 128 net, whose three-plane activations fit the LDS only one row at a time):
    // workgroup blk runs branch blk & 1 of candidate blk >> 1 and writes that branch's eps; the CFG update of the
    // two branches runs as its own launch (unet.hip update_kernel)
    const int brn = R == 1 ? (int)(blk & 1) : 0;
    const int64_t cand0 = R == 1 ? blk >> 1 : blk * RC, row0 = blk * R;
    // the first conv's weights are in flight while x is staged
    prefetch_op<P, R, H, W, 0>(a, __builtin_amdgcn_readfirstlane(tid >> 6), tid & 63, pre);

    // ---- stage x (both branches of each candidate) as 8 zero-padded channels, with its 2 + 5 zero positions
    {
        constexpr CView v = pg.xv;
        constexpr int win = H + 7;
        for (int i = tid; i < R * win; i += FT) {
            const int r = i / win, pw = i - r * win, p = pw - 2;
            const int64_t cand = cand0 + (r < RC ? r : r - RC);
            float xv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (p >= 0 && p < H && cand < a.batch)
                for (int k = 0; k < d; ++k) xv[k] = a.x[((size_t)cand * H + p) * d + k];
            u32x4 o[P];
            split8<P>(f32x4{xv[0], xv[1], xv[2], xv[3]}, f32x4{xv[4], xv[5], xv[6], xv[7]}, o);
#pragma unroll
            for (int pl = 0; pl < P; ++pl)
                *reinterpret_cast<u32x4 *>(sm + v.off + pl * PLB + r * v.rowB + p * v.cs) = o[pl];
        }
    }
    lds_barrier();

    run_ops<P, R, H, W, 0>(a, cand0, row0, brn, pre);

    // ---- the denoise update of this step (or the raw eps of both branches, MODE_EPS)
    const float *E = reinterpret_cast<const float *>(sm + pg.e_off);
    const int flat = H * d, quads = flat / 4;
    if constexpr (R == 1) {  // this row's eps -> eps_c (context branch) / eps_u (masked branch); every mode
        float *out = brn ? a.eps_u : a.eps_c;
        if (cand0 < a.batch)
            for (int i = tid; i < quads; i += FT)
                *reinterpret_cast<f32x4 *>(out + (size_t)cand0 * flat + 4 * i) = *reinterpret_cast<const f32x4 *>(E + 4 * i);
        if constexpr (!PERS) break;
        lds_barrier();
        continue;
    }
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
    if constexpr (!PERS) break;  // one block per workgroup: no loop-carried state (the registers of round 3)
    lds_barrier();  // E (region Z) is read above; the next block stages x into region Z
    }
}

// ---- host

struct Cfg {
    int P, R, H, W;  // numerics planes, rows per workgroup, horizon, waves per workgroup
};
// the instantiated configurations (the LDS of R rows fits one CU: static_assert in the kernel)
// the first match of (P, H) is the default; MPCD_FUSED_ROWS / MPCD_FUSED_WAVES pick another (experiments)
// (1, 2, 64, 4): two or three 4-wave workgroups per CU, their barriers independent (cfg5 14.7 ms per CFG evaluation
// vs 15.3 for one 8-wave workgroup of 4 rows); the split-bf16 nets keep 4-row blocks (their weights, three planes,
// miss the L2 per block: cfg3 3.98 ms with 2-row blocks vs 3.58)
// (3, 1, 128, 8): the fp32-accurate Panda net (H = 128), one row per workgroup, the CFG update as its own launch;
// (2, R, H, 8): the two-term fp16 numerics (MPCD_F16X2) at the f32x3 row counts
#define MPCD_FUSED_CFGS C_(1, 2, 64, 4) C_(3, 4, 32, 8) C_(1, 8, 32, 8) C_(3, 2, 64, 8) C_(1, 2, 128, 8) C_(3, 1, 128, 8) \
    C_(2, 4, 32, 8) C_(2, 2, 64, 8) C_(2, 1, 128, 8) C_(1, 4, 64, 8) C_(1, 2, 64, 8) C_(3, 2, 32, 4)
constexpr Cfg kCfgs[] = {
#define C_(p, r, h, w) {p, r, h, w},
    MPCD_FUSED_CFGS
#undef C_
};

const Prog *prog_of(int P, int R, int H, int W)
{
#define C_(p, r, h, w) \
    if (P == p && R == r && H == h && W == w) return &ProgOf<p, r, h, w>::v;
    MPCD_FUSED_CFGS
#undef C_
    return nullptr;
}

// MPCD_FUSED_PERSIST=1: a grid of (resident workgroups per CU) x CUs walking the row blocks (experiment switch)
bool fused_persistent()
{
    static const bool on = [] {
        const char *e = getenv("MPCD_FUSED_PERSIST");
        return e && e[0] == '1';
    }();
    return on;
}

template <int P, int R, int H, int W>
hipError_t launch_cfg(const FArgs &fa, unsigned grid, hipStream_t st)
{
    constexpr size_t lds = ProgOf<P, R, H, W>::v.lds;
    if (P == 1 || !fused_persistent()) {  // (f16 weights, 2 MB, stay L2-resident: no persistent form)
        constexpr auto kfn = &unet_fused_kernel<P, R, H, W, false>;
        if (hipError_t e = allow_max_lds<kfn>(); e != hipSuccess) return e;
        hipLaunchKernelGGL(kfn, dim3(grid), dim3(64 * W), lds, st, fa);
        return hipGetLastError();
    }
    if constexpr (P != 1) {
        constexpr auto kfn = &unet_fused_kernel<P, R, H, W, true>;
        if (hipError_t e = allow_max_lds<kfn>(); e != hipSuccess) return e;
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(kfn), 64 * W, lds) !=
                hipSuccess || per_cu < 1)
            per_cu = 1;
        const int64_t cap = (int64_t)per_cu * device_cu_count();
        if (cap > 0 && cap < (int64_t)grid) grid = (unsigned)cap;
        hipLaunchKernelGGL(kfn, dim3(grid), dim3(64 * W), lds, st, fa);
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

hipError_t launch_any(int P, int R, int H, int W, const FArgs &fa, unsigned grid, hipStream_t st)
{
#define C_(p, r, h, w) \
    if (P == p && R == r && H == h && W == w) return launch_cfg<p, r, h, w>(fa, grid, st);
    MPCD_FUSED_CFGS
#undef C_
    return hipErrorInvalidValue;
}

}  // namespace

struct UnetFusedPlan {
    int P = 0, R = 0, H = 0, W = 0, d = 0;
    const Prog *prog = nullptr;
    FPtr *ptrs_dev = nullptr;
    ~UnetFusedPlan()
    {
        if (ptrs_dev) (void)hipFree(ptrs_dev);
    }
};

void unet_fused_free(UnetFusedPlan *p) { delete p; }

// Check the compile-time program against the loaded net and build the weight-pointer table; nullptr (and *why)
// when the net or the numerics are not covered (the layer-by-layer path runs it instead).
UnetFusedPlan *unet_fused_prepare(const mpcd_net_desc &d, const UnetWeights &W, int rows_per_wg, std::string *why,
                                  int planes)
{
    auto no = [&](const std::string &m) -> UnetFusedPlan * {
        if (why) *why = m;
        return nullptr;
    };
    if (!W.ready || W.planes == 0) return no("fused U-Net: needs the bf16 / f16 matrix-core numerics");
    const bool h2 = planes ? planes == 2 : W.fused_planes == 2;
    if (planes && planes != 2 && planes != W.planes) return no("fused U-Net: no pack for these numerics");
    if (!d.cfg_masked) return no("fused U-Net: the CFG net (ConditionedTemporalUnet) only");
    if (d.base_dim != 32 || d.n_mults != 3 || d.mults[0] != 1 || d.mults[1] != 2 || d.mults[2] != 4)
        return no("fused U-Net: base 32, dim_mults (1, 2, 4) only");
    if (d.state_dim < 1 || d.state_dim > 8) return no("fused U-Net: state_dim 1..8");
    const int P = h2 ? 2 : W.planes, H = d.horizon;
    if ((H * d.state_dim) % 4) return no("fused U-Net: H*d must be a multiple of 4");
    if (W.n_layers != 35) return no("fused U-Net: unexpected layer count");
    const Prog *pg = nullptr;
    int R = 0, Wv = 0;
    static const int waves = getenv("MPCD_FUSED_WAVES") ? atoi(getenv("MPCD_FUSED_WAVES")) : 0;  // experiments
    for (const Cfg &c : kCfgs)
        if (c.P == P && c.H == H && (rows_per_wg <= 0 || rows_per_wg == c.R) && (waves <= 0 || waves == c.W)) {
            R = c.R;
            Wv = c.W;
            pg = prog_of(c.P, c.R, c.H, c.W);
            break;
        }
    if (!pg) return no("fused U-Net: no instantiation for this horizon / numerics / rows per workgroup");
    std::vector<FPtr> ptrs(pg->n);
    for (int i = 0; i < pg->n; ++i) {
        const COp &o = pg->ops[i];
        const ConvLayer &L = W.layers[o.layer];
        if (o.kind == FK_RESTORE) continue;
        const bool last = o.epi == FE_EPS;
        const bool gn = o.epi == FE_GN || o.epi == FE_GN_COND || o.epi == FE_GN_RES;
        const bool match = L.kind == o.kind && L.cinp8 == o.cinp && L.kc == o.kc &&
                           (last ? L.cout == d.state_dim && L.coutp == 16 : L.cout == o.cout && L.coutp == o.cout) &&
                           (!gn || (L.groups == kGroups && L.gn_w && L.gn_b)) && (o.epi != FE_GN_COND || L.cond_off >= 0);
        if (!match) return no("fused U-Net: layer " + std::to_string(o.layer) + " does not match the program");
        ptrs[i] = FPtr{h2 ? L.wmx2 : L.wmx, L.bias, L.gn_w, L.gn_b, L.cond_off, h2 ? L.inv2 : 1.f};
    }
    auto *pl = new UnetFusedPlan;
    pl->P = P;
    pl->R = R;
    pl->W = Wv;
    pl->H = H;
    pl->d = d.state_dim;
    pl->prog = pg;
    if (hipMalloc(&pl->ptrs_dev, sizeof(FPtr) * ptrs.size()) != hipSuccess ||
        hipMemcpy(pl->ptrs_dev, ptrs.data(), sizeof(FPtr) * ptrs.size(), hipMemcpyHostToDevice) != hipSuccess) {
        delete pl;
        return no("fused U-Net: pointer table upload");
    }
    return pl;
}

// workgroups (row blocks) of one step: R / 2 candidates each, or (R = 1) one branch of one candidate each
static int64_t fused_blocks(const UnetFusedPlan &pl, int64_t batch) { return pl.R == 1 ? 2 * batch : (batch + pl.R / 2 - 1) / (pl.R / 2); }

size_t unet_fused_scratch_bytes(const UnetFusedPlan &pl, int64_t batch)
{
    return (size_t)fused_blocks(pl, batch) * pl.R * pl.prog->skip_elems_per_row * (pl.P == 1 ? 2 : 4);
}

bool unet_fused_split_update(const UnetFusedPlan &pl) { return pl.R == 1; }

int unet_fused_rows_per_wg(const UnetFusedPlan &pl) { return pl.R; }
int unet_fused_planes(const UnetFusedPlan &pl) { return pl.P; }
int unet_fused_waves_per_wg(const UnetFusedPlan &pl) { return pl.W; }
int unet_fused_n_ops(const UnetFusedPlan &pl) { return pl.prog->n; }
int unet_fused_prof_wgs() { return kProfWgs; }
void unet_fused_op_info(const UnetFusedPlan &pl, int i, int32_t out[8])
{
    const COp &o = pl.prog->ops[i];
    const int32_t v[8] = {o.kind, o.epi, o.cinp, o.cout, o.lout, o.kc, 1 << o.ntw_sh, o.ncw};
    for (int k = 0; k < 8; ++k) out[k] = v[k];
}

hipError_t unet_fused_step(const UnetFusedPlan &pl, const UnetFusedStep &s, hipStream_t st)
{
    FArgs fa{};
    fa.ptrs = pl.ptrs_dev;
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
    const int64_t grid = fused_blocks(pl, s.batch);
    if (grid <= 0 || grid > 0x7fffffff) return hipErrorInvalidValue;
    fa.nblk = grid;
    return launch_any(pl.P, pl.R, pl.H, pl.W, fa, (unsigned)grid, st);
}
