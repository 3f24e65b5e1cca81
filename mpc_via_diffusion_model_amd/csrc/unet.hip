// 1D temporal U-Net noise-net + CFG-DDPM / DDIM sampler on gfx950.
//
// Reference: ConditionedTemporalUnet (temporal_unet.py:189-358) / TemporalUnet (:28-187) built from
// ResidualTemporalBlock, Conv1dBlock, Downsample1d, Upsample1d (layers.py:258-355):
//   RTB(x)   = Mish(GN(conv5(Mish(GN(conv5(x))) + cond_j))) + (conv1x1(x) if cin != cout else x)
//   down     = Conv1d k3 s2 p1,  up = ConvTranspose1d k4 s2 p1,  final = Conv1dBlock(k5) -> Conv1d k1
// Activations live in HBM channels-last [row][position][channel]; rows are (branch, candidate):
// for CFG both forwards of p_mean_variance_CFG (diffusion_model_base.py:166-168) run as one batch of
// 2B rows (row < B: context, row >= B: masked context).
//
// Every conv is ONE fused launch (conv_kernel): a workgroup owns `rb` whole rows, stages their input
// window (+halo, zero padded, two tensors for the skip concat) in LDS, runs an implicit GEMM on
// v_mfma_f32_16x16x4_f32 (A = packed weights from L2, B = LDS input columns), then the epilogue
// (bias, GroupNorm over the row's whole group with fp64 statistics, Mish, + cond bias, + residual)
// before one coalesced channels-last store. The denoise update is a separate elementwise kernel.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <vector>

#include "unet.h"

namespace {

thread_local std::string g_unet_err;

int uerr(int code, const std::string &m)
{
    g_unet_err = m;
    return code;
}

enum { CONV_SAME5 = 0, CONV_DOWN3 = 1, CONV_UP4 = 2, CONV_PW1 = 3 };
enum { EPI_BIAS = 0, EPI_GN_MISH = 1, EPI_GN_MISH_COND = 2, EPI_GN_MISH_RES = 3 };
constexpr int CT = 256;  // threads per conv workgroup

struct ConvK {
    const float *xa, *xb;   // inputs [rows_in][lin][ca], [rows_in][lin][cb]
    int ca, cb, cinp, kpad; // channels, padded channels, packed K per parity
    int64_t x_rows;         // rows of xa/xb: row r reads input row r % x_rows
    const float *w;         // packed A operand
    const float *bias;      // [cout]
    const float *gn_w, *gn_b;
    int groups;
    const float *tp;        // tproj row of this step + cond_off (EPI_GN_MISH_COND)
    const float *cp;        // cproj + cond_off or null
    int64_t cp_stride;      // cond_total or 0 (shared context)
    int64_t b_cand;         // candidates per branch (row / b_cand = branch)
    const float *res;       // [rows][lout][cout] (EPI_GN_MISH_RES)
    float *out;             // [rows][lout][cout]
    int64_t rows;
    int lin, lout, cout, coutp;
    int rb;                 // rows per workgroup
    int halo_l, halo_r;     // staged input window = [-halo_l, lin + halo_r)
};

__device__ __forceinline__ f32x4 mfma4c(const f32x4 &w, const f32x4 &a, f32x4 acc)
{
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, a.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, a.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, a.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, a.w, acc, 0, 0, 0);
    return acc;
}

// column c of the workgroup tile -> (local row, output position); false if it is padding
template <int KIND>
__device__ __forceinline__ bool col_pos(const ConvK &a, int c, int &row, int &o, int &par)
{
    if (KIND == CONV_UP4) {
        const int per = a.rb * a.lin, cpar = (per + 15) & ~15;
        par = c / cpar;
        const int rem = c - par * cpar;
        if (par > 1 || rem >= per) return false;
        row = rem / a.lin;
        o = 2 * (rem - row * a.lin) + par;
        return true;
    }
    par = 0;
    if (c >= a.rb * a.lout) return false;
    row = c / a.lout;
    o = c - row * a.lout;
    return true;
}

template <int KIND>
__device__ __forceinline__ int n_cols(const ConvK &a)
{
    if (KIND == CONV_UP4) return 2 * ((a.rb * a.lin + 15) & ~15);
    return a.rb * a.lout;
}

template <int KIND, int EPI>
__device__ __forceinline__ void conv_body(const ConvK &a)
{
    extern __shared__ float sm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t r0 = (int64_t)blockIdx.x * a.rb;
    const int nrow = (int)min((int64_t)a.rb, a.rows - r0);
    const int win = a.lin + a.halo_l + a.halo_r, sin = a.cinp + 4;  // staged input: [rb][win][cinp+4]
    const int ncol = n_cols<KIND>(a), ncol16 = (ncol + 15) & ~15, sout = a.coutp + 4;
    float *s_in = sm;
    float *s_out = s_in + (size_t)a.rb * win * sin;            // [ncol16][coutp+4]
    float *s_stat = s_out + (size_t)ncol16 * sout;             // [rb][groups][2]
    float *s_zero = s_stat + 2 * a.rb * a.groups + 4;          // 4 zeros (padding columns)

    // ---- stage the input window (zero outside [0, lin) and for padded channels / rows)
    const int cin = a.ca + a.cb;
    for (int i = tid; i < a.rb * win * (a.cinp / 4); i += CT) {
        const int q4 = i % (a.cinp / 4), pw = (i / (a.cinp / 4)) % win, r = i / ((a.cinp / 4) * win);
        const int p = pw - a.halo_l, ci = 4 * q4;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (r < nrow && p >= 0 && p < a.lin) {
            const int64_t xr = (r0 + r) % a.x_rows;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = ci + e;
                if (c < a.ca) v[e] = a.xa[((size_t)xr * a.lin + p) * a.ca + c];
                else if (c < cin) v[e] = a.xb[((size_t)xr * a.lin + p) * a.cb + (c - a.ca)];
            }
        }
        *reinterpret_cast<f32x4 *>(s_in + ((size_t)r * win + pw) * sin + ci) = v;
    }
    if (tid < 4) s_zero[tid] = 0.f;
    __syncthreads();

    // ---- implicit GEMM: work item = (16-column tile, pair of 16-channel tiles)
    const int NT = a.coutp / 16, KB = a.kpad / 16, CTL = ncol16 / 16, NP = (NT + 1) / 2;
    const int col_l = lane & 15, q = lane >> 4;
    const int lane16 = lane * 16;
    for (int item = wave; item < CTL * NP; item += CT / 64) {
        const int ctile = item / NP, np = item - ctile * NP;
        const int nt0 = 2 * np, nt1 = min(2 * np + 1, NT - 1);
        const bool two = 2 * np + 1 < NT;
        int row, o, par;
        const bool valid = col_pos<KIND>(a, ctile * 16 + col_l, row, o, par);
        // ctile never straddles an UP parity block (blocks are padded to 16 columns)
        const int tpar = KIND == CONV_UP4 ? ((ctile * 16) / (((a.rb * a.lin) + 15) & ~15)) : 0;
        const uint64_t wa = (uint64_t)(a.w + (size_t)tpar * NT * KB * 256);
        const uint32_t wlo = __builtin_amdgcn_readfirstlane((uint32_t)wa), whi = __builtin_amdgcn_readfirstlane((uint32_t)(wa >> 32));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(((uint64_t)whi << 32) | wlo), (short)0, (int)(NT * KB * 1024), 0x00020000);
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        const float *rowbase = s_in + (size_t)(valid ? row : 0) * win * sin;
#pragma unroll 2
        for (int kb = 0; kb < KB; ++kb) {
            const int k0 = kb * 16 + 4 * q;
            // B operand: input column for (tap / slot, channel quad)
            const float *src;
            if (!valid) {
                src = s_zero;
            } else if (KIND == CONV_UP4) {
                const int slot = k0 / a.cinp, ci0 = k0 - slot * a.cinp;
                const int m = o >> 1;
                const int ip = par == 0 ? (slot == 0 ? m : m - 1) : (slot == 0 ? m + 1 : m);
                src = rowbase + (size_t)(ip + a.halo_l) * sin + ci0;
            } else {
                const int tap = k0 / a.cinp, ci0 = k0 - tap * a.cinp;
                const int ip = KIND == CONV_DOWN3 ? 2 * o + tap - 1 : KIND == CONV_SAME5 ? o + tap - 2 : o;
                src = rowbase + (size_t)(ip + a.halo_l) * sin + ci0;
            }
            const f32x4 b = *reinterpret_cast<const f32x4 *>(src);
            const f32x4 w0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                           rs, lane16, (nt0 * KB + kb) * 1024, 0));
            acc0 = mfma4c(w0, b, acc0);
            if (two) {
                const f32x4 w1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                               rs, lane16, (nt1 * KB + kb) * 1024, 0));
                acc1 = mfma4c(w1, b, acc1);
            }
        }
        // raw conv + bias -> LDS, [column][channel]
        const int c = ctile * 16 + col_l;
        {
            const int n = nt0 * 16 + 4 * q;
            f32x4 v = acc0;
            for (int e = 0; e < 4; ++e) v[e] += n + e < a.cout ? a.bias[n + e] : 0.f;
            *reinterpret_cast<f32x4 *>(s_out + (size_t)c * sout + n) = v;
        }
        if (two) {
            const int n = nt1 * 16 + 4 * q;
            f32x4 v = acc1;
            for (int e = 0; e < 4; ++e) v[e] += n + e < a.cout ? a.bias[n + e] : 0.f;
            *reinterpret_cast<f32x4 *>(s_out + (size_t)c * sout + n) = v;
        }
    }
    __syncthreads();

    // column of (row, o) in s_out
    auto colof = [&](int r, int oo) -> int {
        if (KIND == CONV_UP4) {
            const int p = oo & 1, cpar = ((a.rb * a.lin) + 15) & ~15;
            return p * cpar + r * a.lin + (oo >> 1);
        }
        return r * a.lout + oo;
    };

    // ---- GroupNorm statistics per (row, group), fp64 (torch: biased variance, eps 1e-5)
    if (EPI != EPI_BIAS) {
        const int cpg = a.cout / a.groups;
        for (int sidx = tid; sidx < nrow * a.groups; sidx += CT) {
            const int r = sidx / a.groups, g = sidx - r * a.groups;
            double s1 = 0.0;
            for (int oo = 0; oo < a.lout; ++oo) {
                const float *p = s_out + (size_t)colof(r, oo) * sout + g * cpg;
                for (int cc = 0; cc < cpg; ++cc) s1 += (double)p[cc];
            }
            const double n = (double)cpg * a.lout, mean = s1 / n;
            double s2 = 0.0;
            for (int oo = 0; oo < a.lout; ++oo) {
                const float *p = s_out + (size_t)colof(r, oo) * sout + g * cpg;
                for (int cc = 0; cc < cpg; ++cc) {
                    const double dlt = (double)p[cc] - mean;
                    s2 += dlt * dlt;
                }
            }
            s_stat[2 * sidx] = (float)mean;
            s_stat[2 * sidx + 1] = (float)(1.0 / sqrt(s2 / n + 1e-5));
        }
        __syncthreads();
    }

    // ---- epilogue + store: thread per (row, position, channel quad)
    const int cq = (a.cout + 3) / 4;
    for (int i = tid; i < nrow * a.lout * cq; i += CT) {
        const int q4 = i % cq, oo = (i / cq) % a.lout, r = i / (cq * a.lout);
        const int co = 4 * q4;
        const f32x4 raw = *reinterpret_cast<const f32x4 *>(s_out + (size_t)colof(r, oo) * sout + co);
        const int64_t grow = r0 + r;
        f32x4 v = raw;
        if (EPI != EPI_BIAS) {
            const int cpg = a.cout / a.groups;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int ch = co + e, g = ch / cpg;
                const float mean = s_stat[2 * (r * a.groups + g)], rstd = s_stat[2 * (r * a.groups + g) + 1];
                const float scale = rstd * a.gn_w[ch];
                const float shift = -scale * mean + a.gn_b[ch];
                v[e] = mish(raw[e] * scale + shift);
            }
            if (EPI == EPI_GN_MISH_COND) {
                const int64_t br = grow / a.b_cand, cand = grow - br * a.b_cand;
                f32x4 cv = *reinterpret_cast<const f32x4 *>(a.tp + co);
                if (a.cp && br == 0) cv = cv + *reinterpret_cast<const f32x4 *>(a.cp + (size_t)cand * a.cp_stride + co);
                v = v + cv;
            }
            if (EPI == EPI_GN_MISH_RES)
                v = v + *reinterpret_cast<const f32x4 *>(a.res + ((size_t)grow * a.lout + oo) * a.cout + co);
        }
        float *dst = a.out + ((size_t)grow * a.lout + oo) * a.cout + co;
        if ((a.cout & 3) == 0) {
            *reinterpret_cast<f32x4 *>(dst) = v;
        } else {
            for (int e = 0; e < 4 && co + e < a.cout; ++e) dst[e] = v[e];
        }
    }
}

// the kernel argument reaches the body by reference: it stays in SGPRs, loaded on demand (see unet_mx.hip)
template <int KIND, int EPI>
__global__ __launch_bounds__(CT) void conv_kernel(const ConvK a)
{
    conv_body<KIND, EPI>(a);
}

// x_T into the state (and chain[0])
__global__ void init_x_kernel(float *x, int64_t batch, int flat, const float *noise, uint64_t seed, int64_t goff,
                              float *chain)
{
    const int quads = flat / 4;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= batch * quads) return;
    const int64_t b = i / quads;
    const int qd = (int)(i - b * quads);
    const f32x4 z = noise ? *reinterpret_cast<const f32x4 *>(noise + (size_t)b * flat + 4 * qd)
                          : philox_normal4(seed, (uint64_t)(goff + b), 0u, (uint32_t)qd);
    *reinterpret_cast<f32x4 *>(x + (size_t)b * flat + 4 * qd) = z;
    if (chain) *reinterpret_cast<f32x4 *>(chain + (size_t)b * flat + 4 * qd) = z;
}

// x <- update(x, eps) for one denoise step; same arithmetic as the MLP kernel's update
__global__ void update_kernel(float *x, const float *eps, int64_t batch, int flat, const StepPlan *plan, int s,
                              int mode, int clamp_x0, float wp1, float wf, const float *noise, uint64_t seed,
                              int64_t goff, float *chain, float *x_out, int last, uint32_t *amq)
{
    const int quads = flat / 4;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= batch * quads) return;
    const int64_t b = i / quads;
    const int qd = (int)(i - b * quads);
    const StepPlan sp = plan[s];
    const size_t off = (size_t)b * flat + 4 * qd;
    const f32x4 xv = *reinterpret_cast<const f32x4 *>(x + off);
    const f32x4 ec = *reinterpret_cast<const f32x4 *>(eps + off);
    f32x4 eu = {0.f, 0.f, 0.f, 0.f};
    if (mode != MODE_DDIM) eu = *reinterpret_cast<const f32x4 *>(eps + (size_t)batch * flat + off);
    f32x4 z = {0.f, 0.f, 0.f, 0.f};
    if (mode == MODE_DDPM_CFG && (sp.flags & PLAN_NOISE))
        z = noise ? *reinterpret_cast<const f32x4 *>(noise + (size_t)(s + 1) * batch * flat + off)
                  : philox_normal4(seed, (uint64_t)(goff + b), (uint32_t)(s + 1), (uint32_t)qd);
    const f32x4 o = denoise_update4(sp, mode, clamp_x0, wp1, wf, xv, ec, eu, z);
    *reinterpret_cast<f32x4 *>(x + off) = o;
    if (amq) amq[i] = absmax_bits4(s == 0 ? 0u : amq[i], xv, o);  // running chain |x| maximum of this quad
    if (chain) *reinterpret_cast<f32x4 *>(chain + (size_t)(s + 1) * batch * flat + off) = o;
    if (last && x_out != x) *reinterpret_cast<f32x4 *>(x_out + off) = o;
}

// per-candidate chain |x| maximum from the per-quad running maxima (NaN bits win the integer max)
__global__ void chain_absmax_kernel(const uint32_t *amq, int64_t batch, int quads, float *out)
{
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    uint32_t m = 0;
    for (int q = 0; q < quads; ++q) m = max(m, amq[b * quads + q]);
    out[b] = __builtin_bit_cast(float, m);
}

int group_norm_n_groups(int c)  // layers.py:389-395
{
    if (c < 8) return 1;
    for (int g = 8; g < 18; ++g)
        if (c % g == 0) return g;
    return 1;
}

struct Dims {
    int d, H, base, nres, C;
    std::vector<int> ch;  // channels per level
    int cond_total;
};

Dims dims_of(const mpcd_net_desc &d)
{
    Dims m;
    m.d = d.state_dim;
    m.H = d.horizon;
    m.base = d.base_dim;
    m.nres = d.n_mults;
    m.C = d.context_dim;
    for (int i = 0; i < d.n_mults; ++i) m.ch.push_back(d.base_dim * d.mults[i]);
    return m;
}

int round_up(int v, int m) { return (v + m - 1) / m * m; }

// One packed conv. w_host layout: conv [cout][cin][ks] or convT [cin][cout][4].
int pack_conv(int kind, int cin, int cout, const float *w_host, const float *b_dev, ConvLayer &L,
              std::vector<float> &pack)
{
    L.kind = kind;
    L.cin = cin;
    L.cout = cout;
    L.coutp = round_up(cout, 16);
    L.cinp = round_up(cin, 4);
    const int ks = kind == CONV_SAME5 ? 5 : kind == CONV_DOWN3 ? 3 : kind == CONV_UP4 ? 2 : 1;
    L.kpad = round_up(ks * L.cinp, 16);
    L.bias = b_dev;
    const int npar = kind == CONV_UP4 ? 2 : 1, NT = L.coutp / 16, KB = L.kpad / 16;
    const size_t base = pack.size();
    pack.resize(base + (size_t)npar * NT * KB * 256, 0.f);
    for (int par = 0; par < npar; ++par)
        for (int nt = 0; nt < NT; ++nt)
            for (int kb = 0; kb < KB; ++kb)
                for (int lane = 0; lane < 64; ++lane)
                    for (int s = 0; s < 4; ++s) {
                        const int co = nt * 16 + (lane & 15), k = kb * 16 + 4 * (lane >> 4) + s;
                        const int tap_slot = k / L.cinp, ci = k - tap_slot * L.cinp;
                        float v = 0.f;
                        if (co < cout && ci < cin && tap_slot < ks) {
                            if (kind == CONV_UP4) {
                                // parity 0 (even o): slot0 tap1 (i=m), slot1 tap3 (i=m-1)
                                // parity 1 (odd o):  slot0 tap0 (i=m+1), slot1 tap2 (i=m)
                                const int tap = par == 0 ? (tap_slot == 0 ? 1 : 3) : (tap_slot == 0 ? 0 : 2);
                                v = w_host[((size_t)ci * cout + co) * 4 + tap];
                            } else {
                                v = w_host[((size_t)co * cin + ci) * ks + tap_slot];
                            }
                        }
                        pack[base + ((((size_t)par * NT + nt) * KB + kb) * 64 + lane) * 4 + s] = v;
                    }
    L.w = reinterpret_cast<const float *>(base);  // offset; rebased after upload
    return MPCD_OK;
}

}  // namespace

int unet_prepare(const mpcd_net_desc &d, size_t, const TensorLookup &dev, const TensorLookup &host, UnetWeights &W,
                 void *&pack_dev, size_t &pack_bytes)
{
    W.ready = false;
    W.layers.clear();
    if (d.dtype != MPCD_F32 && d.dtype != MPCD_F32X3 && d.dtype != MPCD_F16 && d.dtype != MPCD_F16X2)
        return uerr(MPCD_EINVAL, "UNet: bad dtype");
    // 0: fp32 MFMA kernels; MPCD_F16X2: the split-bf16 layer-by-layer kernels, the two-term fp16 fused program
    const int planes = (d.dtype == MPCD_F32X3 || d.dtype == MPCD_F16X2) ? 3 : d.dtype == MPCD_F16 ? 1 : 0;
    const bool h2 = d.dtype == MPCD_F16X2;
    std::vector<uint16_t> packmx, packh2;
    if (d.horizon % (1 << (d.n_mults - 1)) != 0) return uerr(MPCD_EINVAL, "UNet: horizon must divide by 2^(levels-1)");
    const Dims m = dims_of(d);
    std::vector<float> pack;
    int cond_off = 0;
    // cond offsets follow the parameter (state_dict) order: downs, ups, mid
    std::vector<std::pair<std::string, int>> cond_cols;
    auto note_cond = [&](const std::string &p, int width) {
        cond_cols.push_back({p, cond_off});
        cond_off += width;
    };
    for (int i = 0; i < m.nres; ++i) {
        note_cond("downs." + std::to_string(i) + ".0", m.ch[i]);
        note_cond("downs." + std::to_string(i) + ".1", m.ch[i]);
    }
    for (int i = 1; i < m.nres; ++i) {
        const int ci = m.ch[m.nres - 1 - i];
        note_cond("ups." + std::to_string(i - 1) + ".0", ci);
        note_cond("ups." + std::to_string(i - 1) + ".1", ci);
    }
    note_cond("mid_block1", m.ch.back());
    note_cond("mid_block2", m.ch.back());
    auto cond_of = [&](const std::string &p) {
        for (auto &c : cond_cols)
            if (c.first == p) return c.second;
        return -1;
    };
    auto need = [&](const std::string &n, const float *p) -> const float * {
        if (!p) g_unet_err = "missing tensor " + n;
        return p;
    };
    int rc = MPCD_OK;
    auto conv = [&](int kind, const std::string &pre, int cin, int cout, bool gn, int cond) {
        ConvLayer L{};
        const float *wh = need(pre + ".weight", host((pre + ".weight").c_str()));
        const float *bd = need(pre + ".bias", dev((pre + ".bias").c_str()));
        if (!wh || !bd) {
            rc = MPCD_EINVAL;
            return;
        }
        pack_conv(kind, cin, cout, wh, bd, L, pack);
        if (planes) unet_pack_mx(kind, cin, cout, planes, wh, L, packmx);
        if (h2) unet_pack_mx(kind, cin, cout, 2, wh, L, packh2);
        L.groups = gn ? group_norm_n_groups(cout) : 1;
        L.cond_off = cond;
        L.gn_w = L.gn_b = nullptr;
        W.layers.push_back(L);
    };
    auto gn_of = [&](const std::string &pre) {
        ConvLayer &L = W.layers.back();
        L.gn_w = need(pre + ".weight", dev((pre + ".weight").c_str()));
        L.gn_b = need(pre + ".bias", dev((pre + ".bias").c_str()));
        if (!L.gn_w || !L.gn_b) rc = MPCD_EINVAL;
    };
    // RTB = [conv1 (+gn, cond)] [res 1x1 if cin != cout] [conv2 (+gn, res)]
    auto rtb = [&](const std::string &p, int cin, int cout) {
        conv(CONV_SAME5, p + ".blocks.0.block.0", cin, cout, true, cond_of(p));
        gn_of(p + ".blocks.0.block.2");
        if (cin != cout) conv(CONV_PW1, p + ".residual_conv", cin, cout, false, -1);
        conv(CONV_SAME5, p + ".blocks.1.block.0", cout, cout, true, -1);
        gn_of(p + ".blocks.1.block.2");
    };
    int prev = m.d;
    for (int i = 0; i < m.nres; ++i) {
        rtb("downs." + std::to_string(i) + ".0", prev, m.ch[i]);
        rtb("downs." + std::to_string(i) + ".1", m.ch[i], m.ch[i]);
        if (i < m.nres - 1) conv(CONV_DOWN3, "downs." + std::to_string(i) + ".4.conv", m.ch[i], m.ch[i], false, -1);
        prev = m.ch[i];
    }
    rtb("mid_block1", m.ch.back(), m.ch.back());
    rtb("mid_block2", m.ch.back(), m.ch.back());
    for (int i = 1; i < m.nres; ++i) {
        const int co = m.ch[m.nres - i], ci = m.ch[m.nres - 1 - i];
        const std::string p = "ups." + std::to_string(i - 1);
        rtb(p + ".0", 2 * co, ci);
        rtb(p + ".1", ci, ci);
        conv(CONV_UP4, p + ".4.conv", ci, ci, false, -1);
    }
    conv(CONV_SAME5, "final_conv.0.block.0", m.base, m.base, true, -1);
    gn_of("final_conv.0.block.2");
    conv(CONV_PW1, "final_conv.1", m.base, m.d, false, -1);
    if (rc) return uerr(rc, g_unet_err);
    if (planes) pack.clear();  // the mx kernels read only their own pack
    const size_t fbytes = (pack.size() * sizeof(float) + 255) / 256 * 256;
    const size_t mxbytes = (packmx.size() * sizeof(uint16_t) + 255) / 256 * 256;
    const size_t bytes = fbytes + mxbytes + packh2.size() * sizeof(uint16_t);
    if (bytes > pack_bytes) {
        if (pack_dev) (void)hipFree(pack_dev);
        pack_dev = nullptr;
        pack_bytes = 0;
        if (hipMalloc(&pack_dev, bytes) != hipSuccess) return uerr(MPCD_ENOMEM, "hipMalloc(unet pack)");
        pack_bytes = bytes;
    }
    if (!pack.empty() && hipMemcpy(pack_dev, pack.data(), pack.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
        return uerr(MPCD_EHIP, "hipMemcpy(unet pack)");
    if (!packmx.empty() && hipMemcpy(static_cast<char *>(pack_dev) + fbytes, packmx.data(),
                                     packmx.size() * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess)
        return uerr(MPCD_EHIP, "hipMemcpy(unet mx pack)");
    if (!packh2.empty() && hipMemcpy(static_cast<char *>(pack_dev) + fbytes + mxbytes, packh2.data(),
                                     packh2.size() * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess)
        return uerr(MPCD_EHIP, "hipMemcpy(unet two-term fp16 pack)");
    for (auto &L : W.layers) {
        L.w = planes ? nullptr : static_cast<const float *>(pack_dev) + reinterpret_cast<size_t>(L.w);
        L.wmx = planes ? reinterpret_cast<const uint16_t *>(static_cast<char *>(pack_dev) + fbytes) +
                             reinterpret_cast<size_t>(L.wmx)
                       : nullptr;
        L.wmx2 = h2 ? reinterpret_cast<const uint16_t *>(static_cast<char *>(pack_dev) + fbytes + mxbytes) +
                          reinterpret_cast<size_t>(L.wmx2)
                    : nullptr;
    }
    W.planes = planes;
    W.fused_planes = h2 ? 2 : 0;
    W.n_layers = (int)W.layers.size();
    W.ready = true;
    W.fused.reset();
    W.fused3.reset();
    W.fused_why.clear();
    // MPCD_FUSED_ROWS=<R>: the fused program with R rows per workgroup (tuning experiments; default: the first
    // instantiated configuration of the net's numerics and horizon)
    static const int fused_rows = getenv("MPCD_FUSED_ROWS") ? atoi(getenv("MPCD_FUSED_ROWS")) : 0;
    if (UnetFusedPlan *fp = unet_fused_prepare(d, W, fused_rows, &W.fused_why)) W.fused.reset(fp, unet_fused_free);
    std::string why3;
    if (h2)
        if (UnetFusedPlan *fp = unet_fused_prepare(d, W, 0, &why3, 3)) W.fused3.reset(fp, unet_fused_free);
    return MPCD_OK;
}

namespace {

// workspace: 6 activation buffers of rows*H*base floats + one skip per level >= 1 + eps
size_t act_floats(const Dims &m, int64_t rows) { return (size_t)rows * m.H * std::max(m.base, m.d); }

struct Buffers {
    float *buf[5];
    std::vector<float *> skip;
    float *eps;
};

Buffers carve(const Dims &m, int64_t rows, void *ws)
{
    Buffers b;
    float *p = static_cast<float *>(ws);
    // per-row footprint of every level is H*base*(mult)/(2^level) <= H*base*max(mult/2^level)
    size_t per = 0;
    for (int i = 0; i < m.nres; ++i) per = std::max(per, (size_t)(m.H >> i) * m.ch[i]);
    per = std::max(per, (size_t)m.H * m.base);
    const size_t n = (size_t)rows * per;
    for (int i = 0; i < 5; ++i) {
        b.buf[i] = p;
        p += n;
    }
    b.skip.assign(m.nres, nullptr);
    for (int i = 1; i < m.nres; ++i) {
        b.skip[i] = p;
        p += (size_t)rows * (m.H >> i) * m.ch[i];
    }
    b.eps = p;
    return b;
}

size_t ws_floats(const Dims &m, int64_t rows)
{
    size_t per = 0;
    for (int i = 0; i < m.nres; ++i) per = std::max(per, (size_t)(m.H >> i) * m.ch[i]);
    per = std::max(per, (size_t)m.H * m.base);
    size_t n = 5 * (size_t)rows * per;
    for (int i = 1; i < m.nres; ++i) n += (size_t)rows * (m.H >> i) * m.ch[i];
    n += (size_t)rows * m.H * m.d + 64;
    return n;
}

struct Ctx {
    const UnetWeights *W;
    int64_t rows, b_cand;
    const float *tp;  // tproj row of this step
    const float *cp;
    int64_t cp_stride;
    hipStream_t st;
    int li;  // next layer index
    // f16 net: activation buffers hold fp16 (halves the activation traffic); the sampler state x
    // (first conv's input) and eps (last conv's output) stay fp32
    bool act_h;
    const float *x_in, *eps_out;
    int act_mask;             // experiment knob (MPCD_UNET_F16_ACT): which buffers are fp16
    const float *hbuf[8];
    bool is_h(const float *p) const
    {
        if (!act_h || !p) return false;
        for (int i = 0; i < 8; ++i)
            if (p == hbuf[i]) return (act_mask >> i) & 1;
        return false;
    }
};

int rows_per_wg(int kind, int lin, int lout, int cinp, int coutp, int halo, size_t &lds)
{
    int rb = std::max(1, (128 + lout - 1) / lout);
    for (; rb >= 1; --rb) {
        const int win = lin + halo;
        const int ncol = kind == CONV_UP4 ? 2 * round_up(rb * lin, 16) : round_up(rb * lout, 16);
        lds = sizeof(float) * ((size_t)rb * win * (cinp + 4) + (size_t)ncol * (coutp + 4) + 2 * rb * 32 + 8);
        if (lds <= 120 * 1024) return rb;
    }
    return 1;
}

template <int KIND, int EPI>
hipError_t launch_conv(const ConvK &k, size_t lds, hipStream_t st)
{
    if (hipError_t e = allow_max_lds<&conv_kernel<KIND, EPI>>(); e != hipSuccess) return e;
    const int64_t blocks = (k.rows + k.rb - 1) / k.rb;
    hipLaunchKernelGGL((conv_kernel<KIND, EPI>), dim3((unsigned)blocks), dim3(CT), lds, st, k);
    return hipGetLastError();
}

hipError_t dispatch(int kind, int epi, const ConvK &k, size_t lds, hipStream_t st)
{
#define CASE(KD, EP) \
    if (kind == KD && epi == EP) return launch_conv<KD, EP>(k, lds, st);
    CASE(CONV_SAME5, EPI_GN_MISH_COND)
    CASE(CONV_SAME5, EPI_GN_MISH_RES)
    CASE(CONV_SAME5, EPI_GN_MISH)
    CASE(CONV_PW1, EPI_BIAS)
    CASE(CONV_DOWN3, EPI_BIAS)
    CASE(CONV_UP4, EPI_BIAS)
#undef CASE
    return hipErrorInvalidValue;
}

// launch parameters of one mx conv (bf16 / f16 MFMA family)
ConvMK make_mk(const Ctx &c, const ConvLayer &L, int epi, const float *xa, int ca, const float *xb, int cb,
               int64_t x_rows, int lin, const float *res, float *out)
{
    ConvMK k{};
    k.xa = xa;
    k.xb = xb;
    k.ca = ca;
    k.cb = cb;
    k.cinp = L.cinp8;
    k.kc = L.kc;
    k.x_rows = x_rows;
    k.w = L.wmx;
    k.bias = L.bias;
    k.gn_w = L.gn_w;
    k.gn_b = L.gn_b;
    k.groups = L.groups;
    k.tp = L.cond_off >= 0 ? c.tp + L.cond_off : nullptr;
    k.cp = (L.cond_off >= 0 && c.cp) ? c.cp + L.cond_off : nullptr;
    k.cp_stride = c.cp_stride;
    k.b_cand = c.b_cand;
    k.res = res;
    k.out = out;
    k.rows = c.rows;
    k.lin = lin;
    k.lout = L.kind == CONV_DOWN3 ? lin / 2 : L.kind == CONV_UP4 ? lin * 2 : lin;
    k.cout = L.cout;
    k.coutp = L.coutp;
    k.epi = epi;
    k.in_h = c.is_h(xa);
    k.res_h = c.is_h(res);
    k.out_h = c.is_h(out);
    k.layer = (int)(&L - c.W->layers.data());
    return k;
}

// out = layer(xa [, xb]); lin = input length
int run_conv(Ctx &c, int epi, const float *xa, int ca, const float *xb, int cb, int64_t x_rows, int lin,
             const float *res, float *out)
{
    const ConvLayer &L = c.W->layers[c.li++];
    if (L.cin != ca + cb) return uerr(MPCD_EINVAL, "UNet plan: channel mismatch");
    if (c.W->planes) {
        ConvMK k = make_mk(c, L, epi, xa, ca, xb, cb, x_rows, lin, res, out);
        if (epi == EPI_GN_MISH_COND && !k.tp) return uerr(MPCD_EINVAL, "UNet plan: missing cond");
        if (L.cout % L.groups != 0) return uerr(MPCD_EUNSUP, "UNet: cout not divisible by groups");
        std::string why;
        hipError_t e = unet_launch_mx(L.kind, c.W->planes, k, c.st, &why);
        if (e != hipSuccess) return uerr(MPCD_EHIP, "mx conv launch: " + (why.empty() ? hipGetErrorString(e) : why));
        return MPCD_OK;
    }
    ConvK k{};
    k.xa = xa;
    k.xb = xb;
    k.ca = ca;
    k.cb = cb;
    k.cinp = L.cinp;
    k.kpad = L.kpad;
    k.x_rows = x_rows;
    k.w = L.w;
    k.bias = L.bias;
    k.gn_w = L.gn_w;
    k.gn_b = L.gn_b;
    k.groups = L.groups;
    k.tp = L.cond_off >= 0 ? c.tp + L.cond_off : nullptr;
    k.cp = (L.cond_off >= 0 && c.cp) ? c.cp + L.cond_off : nullptr;
    k.cp_stride = c.cp_stride;
    k.b_cand = c.b_cand;
    k.res = res;
    k.out = out;
    k.rows = c.rows;
    k.lin = lin;
    k.lout = L.kind == CONV_DOWN3 ? lin / 2 : L.kind == CONV_UP4 ? lin * 2 : lin;
    k.cout = L.cout;
    k.coutp = L.coutp;
    const int taps = L.kpad / L.cinp;  // padded taps (zero weights beyond the real ones)
    if (L.kind == CONV_SAME5) {
        k.halo_l = 2;
        k.halo_r = std::max(2, taps - 3);
    } else if (L.kind == CONV_DOWN3) {
        k.halo_l = 1;
        k.halo_r = std::max(1, taps - 2);
    } else if (L.kind == CONV_UP4) {
        k.halo_l = 1;
        k.halo_r = 1;
    } else {
        k.halo_l = 0;
        k.halo_r = std::max(0, taps - 1);
    }
    size_t lds = 0;
    k.rb = rows_per_wg(L.kind, lin, k.lout, L.cinp, L.coutp, k.halo_l + k.halo_r, lds);
    if (epi == EPI_GN_MISH_COND && !k.tp) return uerr(MPCD_EINVAL, "UNet plan: missing cond");
    if (L.cout % L.groups != 0) return uerr(MPCD_EUNSUP, "UNet: cout not divisible by groups");
    hipError_t e = dispatch(L.kind, epi, k, lds, c.st);
    if (e != hipSuccess) return uerr(MPCD_EHIP, std::string("conv launch: ") + hipGetErrorString(e));
    return MPCD_OK;
}

// ResidualTemporalBlock: x (+ xb concat) at length L -> out
int run_rtb(Ctx &c, Buffers &B, const float *xa, int ca, const float *xb, int cb, int64_t x_rows, int L, int cout,
            float *tmp_h, float *tmp_r, float *out)
{
    int rc;
    if (c.W->planes) {  // mx family: [residual 1x1 conv], then conv1 + conv2 (fused when that measures faster)
        const ConvLayer &L1 = c.W->layers[c.li];
        const bool has_res = ca + cb != cout;
        const ConvLayer &L2 = c.W->layers[c.li + (has_res ? 2 : 1)];
        if (L1.cin != ca + cb || L2.cin != cout || L1.cout != cout || L2.cout != cout)
            return uerr(MPCD_EINVAL, "UNet plan: channel mismatch");
        const float *res = xa;
        if (has_res) {
            c.li += 1;
            if ((rc = run_conv(c, EPI_BIAS, xa, ca, xb, cb, x_rows, L, nullptr, tmp_r))) return rc;
            c.li -= 2;
            res = tmp_r;
        } else if (x_rows != c.rows) {
            return uerr(MPCD_EUNSUP, "UNet: identity residual on shared input");
        }
        ConvMK k1 = make_mk(c, L1, EPI_GN_MISH_COND, xa, ca, xb, cb, x_rows, L, nullptr, tmp_h);
        ConvMK k2 = make_mk(c, L2, EPI_GN_MISH_RES, tmp_h, cout, nullptr, 0, c.rows, L, res, out);
        c.li += has_res ? 3 : 2;
        if (!k1.tp) return uerr(MPCD_EINVAL, "UNet plan: missing cond");
        if (L1.cout % L1.groups != 0 || L2.cout % L2.groups != 0)
            return uerr(MPCD_EUNSUP, "UNet: cout not divisible by groups");
        std::string why;
        hipError_t e = unet_launch_mx_rtb(c.W->planes, k1, k2, c.st, &why);
        if (e != hipSuccess) return uerr(MPCD_EHIP, "mx block launch: " + (why.empty() ? hipGetErrorString(e) : why));
        return MPCD_OK;
    }
    if ((rc = run_conv(c, EPI_GN_MISH_COND, xa, ca, xb, cb, x_rows, L, nullptr, tmp_h))) return rc;
    const float *res = xa;
    if (ca + cb != cout) {
        if ((rc = run_conv(c, EPI_BIAS, xa, ca, xb, cb, x_rows, L, nullptr, tmp_r))) return rc;
        res = tmp_r;
    } else if (x_rows != c.rows) {
        return uerr(MPCD_EUNSUP, "UNet: identity residual on shared input");
    }
    return run_conv(c, EPI_GN_MISH_RES, tmp_h, cout, nullptr, 0, c.rows, L, res, out);
}

// one full noise-net forward: x [b_cand][H][d] (shared by the branches) -> eps [rows][H][d]
int forward(Ctx &c, const Dims &m, Buffers &B, const float *x, int64_t x_rows)
{
    int rc;
    c.li = 0;
    c.x_in = x;
    c.eps_out = B.eps;
    for (int i = 0; i < 5; ++i) c.hbuf[i] = B.buf[i];
    for (int i = 0; i < 3; ++i) c.hbuf[5 + i] = i + 1 < (int)B.skip.size() ? B.skip[i + 1] : nullptr;
    float *A = B.buf[0], *Bb = B.buf[1], *T = B.buf[2], *R = B.buf[3], *D = B.buf[4];
    const float *cur = x;
    int cc = m.d, L = m.H;
    int64_t cur_rows = x_rows;
    for (int i = 0; i < m.nres; ++i) {
        const int co = m.ch[i];
        if ((rc = run_rtb(c, B, cur, cc, nullptr, 0, cur_rows, L, co, T, R, A))) return rc;
        float *skip = i >= 1 ? B.skip[i] : Bb;
        if ((rc = run_rtb(c, B, A, co, nullptr, 0, c.rows, L, co, T, R, skip))) return rc;
        cur = skip;
        cur_rows = c.rows;
        cc = co;
        if (i < m.nres - 1) {
            if ((rc = run_conv(c, EPI_BIAS, skip, co, nullptr, 0, c.rows, L, nullptr, D))) return rc;
            L /= 2;
            cur = D;
        }
    }
    // mid
    if ((rc = run_rtb(c, B, cur, cc, nullptr, 0, c.rows, L, cc, T, R, A))) return rc;
    if ((rc = run_rtb(c, B, A, cc, nullptr, 0, c.rows, L, cc, T, R, Bb))) return rc;
    cur = Bb;
    // ups: cur is Bb (mid) or D (previous up); RTB1 -> A, RTB2 -> Bb (cur is dead once RTB1's conv1 and
    // residual conv have read it), up-conv -> D
    for (int i = 1; i < m.nres; ++i) {
        const int co = m.ch[m.nres - i], ci = m.ch[m.nres - 1 - i];
        const float *skip = B.skip[m.nres - i];
        if ((rc = run_rtb(c, B, cur, co, skip, co, c.rows, L, ci, T, R, A))) return rc;
        if ((rc = run_rtb(c, B, A, ci, nullptr, 0, c.rows, L, ci, T, R, Bb))) return rc;
        if ((rc = run_conv(c, EPI_BIAS, Bb, ci, nullptr, 0, c.rows, L, nullptr, D))) return rc;
        L *= 2;
        cur = D;
        cc = ci;
    }
    if ((rc = run_conv(c, EPI_GN_MISH, cur, cc, nullptr, 0, c.rows, L, nullptr, T))) return rc;
    return run_conv(c, EPI_BIAS, T, m.base, nullptr, 0, c.rows, L, nullptr, B.eps);
}

}  // namespace

namespace {
std::atomic<int> g_unet_path{0};  // mpcd_unet_force_path

// the fused form runs the CFG samplers and the two-branch eps of a ConditionedTemporalUnet it covers;
// MPCD_UNET_FUSED=0 turns it off (the layer-by-layer path then runs everything)
// the fused program a sampler mode runs: an MPCD_F16X2 net's unclamped DDIM samplers take its split-bf16 program
const UnetFusedPlan *fused_plan(const UnetWeights &W, int mode)
{
    if (W.fused_planes == 2 && (W.force3 || mode == MODE_DDIM_CFG || mode == MODE_DDIM)) return W.fused3.get();
    return W.fused.get();
}

bool use_fused(const UnetWeights &W, int mode)
{
    static const bool env_off = [] {
        const char *e = getenv("MPCD_UNET_FUSED");
        return e && e[0] == '0';
    }();
    const int path = g_unet_path.load();
    if (!fused_plan(W, mode) || path == 1 || (env_off && path != 2)) return false;
    return mode == MODE_DDPM_CFG || mode == MODE_DDIM_CFG || mode == MODE_EPS;
}
}  // namespace

void unet_force_path(int path) { g_unet_path.store(path); }

bool unet_use_fused(const UnetWeights &W, int mode) { return use_fused(W, mode); }

void unet_form(const UnetWeights &W, int mode, int32_t out[4])
{
    const bool f = use_fused(W, mode);
    out[0] = f ? 1 : 0;
    const UnetFusedPlan *pl = fused_plan(W, mode);
    out[1] = f ? unet_fused_planes(*pl) : W.planes;
    out[2] = f ? unet_fused_rows_per_wg(*pl) : 0;
    out[3] = f ? unet_fused_waves_per_wg(*pl) : 0;
}

size_t unet_workspace_bytes(const mpcd_net_desc &d, const UnetWeights &W, bool fused, int64_t batch, int nb)
{
    const Dims m = dims_of(d);
    // + the sampler state x [B][H][d] and the per-quad chain |x| maxima [B][H*d/4]
    const size_t state = sizeof(float) * ((size_t)batch * m.H * m.d + (size_t)batch * (m.H * m.d / 4 + 1));
    if (fused)  // + the eps of both branches when the update is its own launch (unet_fused_split_update)
    {
        size_t mx = 0;  // the larger of the net's fused programs (an MPCD_F16X2 net has two)
        for (const UnetFusedPlan *pl : {W.fused.get(), W.fused3.get()})
            if (pl)
                mx = std::max(mx, unet_fused_scratch_bytes(*pl, batch) +
                                      (unet_fused_split_update(*pl) ? sizeof(float) * 2 * (size_t)batch * m.H * m.d + 256 : 0));
        return state + 256 + mx;
    }
    return sizeof(float) * ws_floats(m, batch * nb) + state;
}

namespace {
// the whole net + the update of one denoise step per launch (unet_fused.hip)
int sample_fused(const mpcd_net_desc &d, const UnetWeights &W, const UnetSampleArgs &a, hipStream_t st)
{
    const UnetFusedPlan &pl = *fused_plan(W, a.mode);
    const int flat = d.horizon * d.state_dim;
    float *xs = static_cast<float *>(a.workspace);
    uint32_t *amq = a.chain_absmax ? reinterpret_cast<uint32_t *>(xs + (size_t)a.batch * flat) : nullptr;
    char *scratch = reinterpret_cast<char *>(xs) +
                    ((sizeof(float) * ((size_t)a.batch * flat + (size_t)a.batch * (flat / 4 + 1)) + 255) / 256 * 256);
    UnetFusedStep f{};
    f.batch = a.batch;
    f.goff = a.global_offset;
    f.mode = a.mode;
    f.clamp_x0 = a.clamp_x0;
    f.cp = a.cproj;
    f.cp_stride = a.cproj_stride;
    f.plan = a.plan;
    f.wp1 = a.wp1;
    f.wf = a.wf;
    f.noise = a.noise;
    f.seed = a.seed;
    f.chain = a.chain;
    f.x_out = a.x_out;
    f.amq = amq;
    f.scratch = scratch;
    const bool split = unet_fused_split_update(pl);
    float *eps_buf = split ? reinterpret_cast<float *>(scratch + (unet_fused_scratch_bytes(pl, a.batch) + 255) / 256 * 256)
                           : nullptr;
    if (a.mode == MODE_EPS) {
        f.x = const_cast<float *>(a.x_in);  // read only in MODE_EPS
        f.tp = a.tproj;
        f.eps_c = a.eps_cond;
        f.eps_u = a.eps_uncond;
        f.chain = f.x_out = nullptr;
        f.amq = nullptr;
        hipError_t e = unet_fused_step(pl, f, st);
        return e == hipSuccess ? MPCD_OK : uerr(MPCD_EHIP, std::string("fused U-Net: ") + hipGetErrorString(e));
    }
    const int threads = 256;
    const unsigned g1 = (unsigned)((a.batch * (flat / 4) + threads - 1) / threads);
    hipLaunchKernelGGL(init_x_kernel, dim3(g1), dim3(threads), 0, st, xs, a.batch, flat, a.noise, a.seed,
                       a.global_offset, a.chain);
    f.x = xs;
    // diagnostics: MPCD_FUSED_PROF=<file> writes the per-op s_memtime stamps of the third step's first workgroups
    static const char *prof_path = getenv("MPCD_FUSED_PROF");
    uint64_t *prof = nullptr;
    const size_t prof_n = (size_t)unet_fused_prof_wgs() * unet_fused_n_ops(pl) * 4;
    if (prof_path && a.n_steps > 2 && hipMalloc(&prof, prof_n * 8) == hipSuccess) (void)hipMemsetAsync(prof, 0, prof_n * 8, st);
    for (int s = 0; s < a.n_steps; ++s) {
        f.tp = a.tproj + (size_t)s * a.cond_total;
        f.step = s;
        f.last = s == a.n_steps - 1 ? 1 : 0;
        f.prof = s == 2 ? prof : nullptr;
        if (split) {
            f.eps_c = eps_buf;
            f.eps_u = eps_buf + (size_t)a.batch * flat;
        }
        hipError_t e = unet_fused_step(pl, f, st);
        if (e != hipSuccess) return uerr(MPCD_EHIP, std::string("fused U-Net: ") + hipGetErrorString(e));
        if (split) {
            hipLaunchKernelGGL(update_kernel, dim3(g1), dim3(threads), 0, st, xs, eps_buf, a.batch, flat, a.plan, s, a.mode,
                               a.clamp_x0, a.wp1, a.wf, a.noise, a.seed, a.global_offset, a.chain, a.x_out,
                               s == a.n_steps - 1 ? 1 : 0, amq);
            if ((e = hipGetLastError()) != hipSuccess)
                return uerr(MPCD_EHIP, std::string("fused U-Net update: ") + hipGetErrorString(e));
        }
    }
    if (prof) {
        std::vector<uint64_t> h(prof_n);
        if (hipStreamSynchronize(st) == hipSuccess && hipMemcpy(h.data(), prof, prof_n * 8, hipMemcpyDeviceToHost) == hipSuccess)
            if (FILE *fp = fopen(prof_path, "wb")) {
                const int32_t hdr[2] = {unet_fused_prof_wgs(), unet_fused_n_ops(pl)};
                fwrite(hdr, 4, 2, fp);
                fwrite(h.data(), 8, h.size(), fp);
                for (int i = 0; i < unet_fused_n_ops(pl); ++i) {
                    int32_t info[8];
                    unet_fused_op_info(pl, i, info);
                    fwrite(info, 4, 8, fp);
                }
                fclose(fp);
            }
        (void)hipFree(prof);
    }
    if (amq)
        hipLaunchKernelGGL(chain_absmax_kernel, dim3((unsigned)((a.batch + 255) / 256)), dim3(256), 0, st, amq, a.batch,
                           flat / 4, a.chain_absmax);
    if (hipGetLastError() != hipSuccess) return uerr(MPCD_EHIP, "fused U-Net: update launch");
    return MPCD_OK;
}
}  // namespace

int unet_sample(const mpcd_net_desc &d, const UnetWeights &W, const UnetSampleArgs &a, hipStream_t st)
{
    if (!W.ready) return uerr(MPCD_ESTATE, "UNet weights not prepared");
    if (a.fused) {
        if (!fused_plan(W, a.mode)) return uerr(MPCD_EUNSUP, "fused U-Net form requested but not prepared: " + W.fused_why);
        return sample_fused(d, W, a, st);
    }
    if (g_unet_path.load() == 2)  // forced fused, and unet_use_fused said no
        return uerr(MPCD_EUNSUP, "fused U-Net forced but not applicable: " +
                                     (W.fused ? std::string("sampler mode") : W.fused_why));
    const Dims m = dims_of(d);
    const bool eps_mode = a.mode == MODE_EPS || a.mode == MODE_EPS1;
    const int nb = (a.mode == MODE_DDIM || a.mode == MODE_EPS1) ? 1 : 2;
    const int64_t rows = a.batch * nb;
    Buffers B = carve(m, rows, a.workspace);
    float *xs = static_cast<float *>(a.workspace) + ws_floats(m, rows);  // sampler state [B][H][d]
    const int flat = m.H * m.d;
    if (flat % 4) return uerr(MPCD_EUNSUP, "UNet sampler: H*d must be a multiple of 4");
    Ctx c{};
    c.W = &W;
    c.rows = rows;
    c.b_cand = a.batch;
    c.cp = a.cproj;
    c.cp_stride = a.cproj_stride;
    c.st = st;
    {
        const char *e = getenv("MPCD_UNET_F16_ACT");  // experiment knob: 0 keeps fp32 activations
        c.act_mask = e && e[0] ? atoi(e) : 255;
        c.act_h = W.planes == 1 && c.act_mask != 0;
    }
    const int threads = 256;
    const int64_t nq = a.batch * (flat / 4);
    const unsigned g1 = (unsigned)((nq + threads - 1) / threads);
    if (eps_mode) {
        c.tp = a.tproj;
        int rc = forward(c, m, B, a.x_in, a.batch);
        if (rc) return rc;
        if (hipMemcpyAsync(a.eps_cond, B.eps, sizeof(float) * a.batch * flat, hipMemcpyDeviceToDevice, st) != hipSuccess)
            return uerr(MPCD_EHIP, "copy eps");
        if (nb == 2 && hipMemcpyAsync(a.eps_uncond, B.eps + (size_t)a.batch * flat, sizeof(float) * a.batch * flat,
                                      hipMemcpyDeviceToDevice, st) != hipSuccess)
            return uerr(MPCD_EHIP, "copy eps");
        return MPCD_OK;
    }
    uint32_t *amq = a.chain_absmax ? reinterpret_cast<uint32_t *>(xs + (size_t)a.batch * flat) : nullptr;
    hipLaunchKernelGGL(init_x_kernel, dim3(g1), dim3(threads), 0, st, xs, a.batch, flat, a.noise, a.seed,
                       a.global_offset, a.chain);
    for (int s = 0; s < a.n_steps; ++s) {
        c.tp = a.tproj + (size_t)s * a.cond_total;
        int rc = forward(c, m, B, xs, a.batch);
        if (rc) return rc;
        hipLaunchKernelGGL(update_kernel, dim3(g1), dim3(threads), 0, st, xs, B.eps, a.batch, flat, a.plan, s, a.mode,
                           a.clamp_x0, a.wp1, a.wf, a.noise, a.seed, a.global_offset, a.chain, a.x_out,
                           s == a.n_steps - 1 ? 1 : 0, amq);
    }
    if (amq)
        hipLaunchKernelGGL(chain_absmax_kernel, dim3((unsigned)((a.batch + 255) / 256)), dim3(256), 0, st, amq, a.batch,
                           flat / 4, a.chain_absmax);
    if (hipGetLastError() != hipSuccess) return uerr(MPCD_EHIP, "update launch");
    return MPCD_OK;
}

const char *unet_last_error() { return g_unet_err.c_str(); }
