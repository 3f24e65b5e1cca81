// Native training step for the CFG MLP noise-net: GaussianDiffusionModel.p_losses
// with CFG context dropout (mpd/models/diffusion_models/diffusion_model_base.py:434-467), the WeightedL2
// loss (helpers.py:71-99), backward through every layer, torch.optim.Adam (trainer.py:152) and the
// EMA model update (trainer.py:70-88, 302-308), all on the device in fp32.
//
// Training is offline and sized by the training batch (thousands of rows, widths <= 256), so the
// GEMMs are one LDS-tiled fp32 kernel with generic operand strides (Y = X W^T, dX = dY W, dW = dY^T X
// and the bias gradients as dY^T 1), and everything else is elementwise. Activations of the forward
// pass stay in HBM for the backward pass ([rows][width] row-major, one buffer per tensor).
//
// Net (oracle/nets.py ConditionedMLPNet = temporal_unet.py PointUnet stack with a CFG context):
//   t_emb = L_t2(Mish(L_t1(sinemb(t))));  c = cat(t_emb, ctx * (1 - mask));  mc = Mish(c)
//   block(x) = Mish(L_b(Mish(L_a x)) + L_c mc)      (TemporalBlockMLP, layers.py:358-385)
//   downs d0..d{n-1}, mid, ups u_k(cat(y, d_{n-2-k})), out = L_f2(L_f1 y)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

#include "comm.h"
#include "train.h"

namespace {

constexpr int GT = 64;   // GEMM tile (rows and columns of C per workgroup)
constexpr int GK = 16;   // k-step staged in LDS

// rs (optional, the column-0 workgroups): rs[z*M + m] = sum_k A(m,k) over the slice, in k order, from the staged A
// tile — for dW = dY^T X that is the bias gradient's slice of dY's column sums, without a second pass over dY.
MPCD_DEV float rowsum_step(const float (&As)[GK][GT + 1], float acc)
{
#pragma unroll
    for (int kk = 0; kk < GK; ++kk) acc += As[kk][threadIdx.x];
    return acc;
}

// C[m][n] (ldc) = beta * C + sum_k A(m,k) B(k,n) (+ bias[n]); A(m,k) = a[m*sam + k*sak], B(k,n) = b[k*sbk + n*sbn].
// 256 threads, each a 4x4 block of C; the k-sum runs in k order per output (fp32 FMA off: -ffp-contract=off).
// Split K (gridDim.z > 1): slice z sums k in [z*kchunk, (z+1)*kchunk) into c + z*zstride (beta 0, no bias);
// splitk_reduce_kernel then adds the slices in z order (deterministic).
__global__ __launch_bounds__(256) void gemm_kernel(int M, int N, int K, const float *__restrict__ a, int64_t sam,
                                                   int64_t sak, const float *__restrict__ b, int64_t sbk, int64_t sbn,
                                                   float *__restrict__ c, int64_t ldc, float beta,
                                                   const float *__restrict__ bias, int kchunk, int64_t zstride,
                                                   float *__restrict__ rs)
{
    __shared__ float As[GK][GT + 1], Bs[GK][GT + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
    const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
    c += blockIdx.z * zstride;
    float acc[4][4] = {};
    const bool rsum = rs && blockIdx.x == 0 && threadIdx.x < GT;
    float rsacc = 0.f;
    for (int k0 = kb; k0 < ke; k0 += GK) {
        for (int i = threadIdx.x; i < GK * GT; i += 256) {
            const int kk = i / GT, r = i % GT;
            const int m = m0 + r, n = n0 + r, k = k0 + kk;
            As[kk][r] = (m < M && k < ke) ? a[m * sam + k * sak] : 0.f;
            Bs[kk][r] = (n < N && k < ke) ? b[k * sbk + n * sbn] : 0.f;
        }
        __syncthreads();
        if (rsum) rsacc = rowsum_step(As, rsacc);
#pragma unroll
        for (int kk = 0; kk < GK; ++kk) {
            float av[4], bv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                av[i] = As[kk][ty + 16 * i];
                bv[i] = Bs[kk][tx + 16 * i];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] += av[i] * bv[j];
        }
        __syncthreads();
    }
    if (rsum && m0 + (int)threadIdx.x < M) rs[blockIdx.z * (int64_t)M + m0 + threadIdx.x] = rsacc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + ty + 16 * i;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + tx + 16 * j;
            if (n >= N) continue;
            float v = acc[i][j];
            if (bias) v += bias[n];
            float *p = c + m * ldc + n;
            *p = beta != 0.f ? *p + v : v;
        }
    }
}

// The same contract on the fp32 matrix cores: v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulate).
// 4 waves, each a 32x32 quarter of the 64x64 tile as 2x2 MFMA tiles; the LDS staging is gemm_kernel's.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void gemm_mfma_kernel(int M, int N, int K, const float *__restrict__ a, int64_t sam,
                                                        int64_t sak, const float *__restrict__ b, int64_t sbk,
                                                        int64_t sbn, float *__restrict__ c, int64_t ldc, float beta,
                                                        const float *__restrict__ bias, int kchunk, int64_t zstride,
                                                        float *__restrict__ rs)
{
    __shared__ float As[GK][GT + 1], Bs[GK][GT + 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
    const int r16 = lane & 15, kq = lane >> 4;
    const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
    const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
    c += blockIdx.z * zstride;
    f32x4_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const bool rsum = rs && blockIdx.x == 0 && threadIdx.x < GT;
    float rsacc = 0.f;
    // register double buffer: the next k-step's operands are loaded while this one's MFMAs run
    constexpr int PT = GK * GT / 256;
    const int sr = threadIdx.x % GT, sk = threadIdx.x / GT;
    const bool mok = m0 + sr < M, nok = n0 + sr < N;
    const float *ap = a + (m0 + sr) * sam, *bp = b + (n0 + sr) * sbn;
    float ra[PT], rb[PT];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const int k = k0 + sk + j * (256 / GT);
            ra[j] = (mok && k < ke) ? ap[k * sak] : 0.f;
            rb[j] = (nok && k < ke) ? bp[k * sbk] : 0.f;
        }
    };
    fetch(kb);
    for (int k0 = kb; k0 < ke; k0 += GK) {
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            As[sk + j * (256 / GT)][sr] = ra[j];
            Bs[sk + j * (256 / GT)][sr] = rb[j];
        }
        __syncthreads();
        if (k0 + GK < ke) fetch(k0 + GK);
        if (rsum) rsacc = rowsum_step(As, rsacc);
#pragma unroll
        for (int kk = 0; kk < GK; kk += 4) {
            float af[2], bf[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                af[t] = As[kk + kq][wm + t * 16 + r16];
                bf[t] = Bs[kk + kq][wn + t * 16 + r16];
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    if (rsum && m0 + (int)threadIdx.x < M) rs[blockIdx.z * (int64_t)M + m0 + threadIdx.x] = rsacc;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int m = m0 + wm + i * 16 + 4 * kq + e, n = n0 + wn + j * 16 + r16;
                if (m >= M || n >= N) continue;
                float v = acc[i][j][e];
                if (bias) v += bias[n];
                float *p = c + m * ldc + n;
                *p = beta != 0.f ? *p + v : v;
            }
}

// sum_{z < Z} p[z * stride], added in z order (deterministic) with 8 loads in flight
MPCD_DEV float sum_slices(const float *p, int64_t stride, int Z)
{
    float acc = 0.f;
    int z = 0;
    for (; z + 8 <= Z; z += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[(z + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; z < Z; ++z) acc += p[z * stride];
    return acc;
}

// C[m][n] = beta * C + sum_z part[z][m][n] (+ bias[n])
__global__ void splitk_reduce_kernel(int M, int N, int Z, const float *part, float *c, int64_t ldc, float beta,
                                     const float *bias)
{
    const int64_t n = (int64_t)M * N;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float acc = sum_slices(part + i, n, Z);
        const int m = (int)(i / N), j = (int)(i - (int64_t)m * N);
        if (bias) acc += bias[j];
        float *p = c + m * ldc + j;
        *p = beta != 0.f ? *p + acc : acc;
    }
}

// column sums over a row slice: part[z][n] = sum_{m in slice z} dy[m*ld + n]
__global__ __launch_bounds__(256) void colsum_part_kernel(int64_t M, int N, const float *dy, int64_t ld, int64_t rchunk,
                                                          float *part)
{
    __shared__ float s[4][64];
    const int c = threadIdx.x & 63, r = threadIdx.x >> 6, n = blockIdx.x * 64 + c;
    const int64_t mb = blockIdx.y * rchunk, me = min(M, mb + rchunk);
    float acc = 0.f;
    if (n < N)
        for (int64_t m0 = mb + r; m0 < me; m0 += 4 * 8) {  // 8 independent loads in flight, summed in order
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t m = m0 + 4 * u;
                v[u] = m < me ? dy[m * ld + n] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
    s[r][c] = acc;
    __syncthreads();
    if (r == 0 && n < N) part[blockIdx.y * (int64_t)N + n] = (s[0][c] + s[1][c]) + (s[2][c] + s[3][c]);
}

// db[n] += sum_z part[z][n]
__global__ void colsum_reduce_kernel(int N, int Z, const float *part, float *db)
{
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    db[n] += sum_slices(part + n, N, Z);
}

MPCD_DEV float softplus(float x) { return log1pf(expf(x)); }  // as torch's Mish kernels (no threshold)

// Mish forward (torch: x * tanh(softplus(x)))
__global__ void mish_fwd_kernel(int64_t n, const float *__restrict__ pre, float *__restrict__ out)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = pre[i] * tanhf(softplus(pre[i]));
}

// d pre (+)= d out * (tanh(sp) + x * sigmoid(x) * (1 - tanh(sp)^2))  (torch's Mish backward); in place allowed
__global__ void mish_bwd_kernel(int64_t n, const float *__restrict__ pre, const float *dout, float *dpre, int acc)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float x = pre[i];
        const float tsp = tanhf(softplus(x));
        const float sg = 1.f / (1.f + expf(-x));
        const float d = dout[i] * (tsp + x * sg * (1.f - tsp * tsp));
        dpre[i] = acc ? dpre[i] + d : d;
    }
}

// ---- U-Net trunk ops, channels-last [b][l][c]

// col[(b*Lout + o)][ci*k + tap] = x(b, o*s - p + tap, ci), ci < ca from xa, else from xb (channel concat)
__global__ void im2col_kernel(int64_t B, int Lin, int Lout, int ca, int cb, int k, int s, int p, const float *xa,
                              const float *xb, float *col)
{
    const int cin = ca + cb, W = cin * k;
    const int64_t n = B * Lout * W;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / W;
        const int j = (int)(i - r * W), ci = j / k, tap = j - ci * k;
        const int64_t b = r / Lout;
        const int o = (int)(r - b * Lout), pos = o * s - p + tap;
        float v = 0.f;
        if (pos >= 0 && pos < Lin)
            v = ci < ca ? xa[(b * Lin + pos) * ca + ci] : xb[(b * Lin + pos) * cb + (ci - ca)];
        col[i] = v;
    }
}

// dx(b, i, ci) += sum over (o, tap) with o*s - p + tap = i of dcol[(b*Lout + o)][ci*k + tap]  (gather, no atomics)
__global__ void col2im_kernel(int64_t B, int Lin, int Lout, int ca, int cb, int k, int s, int p, const float *dcol,
                              float *dxa, float *dxb)
{
    const int cin = ca + cb, W = cin * k;
    const int64_t n = B * Lin * cin;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / cin;
        const int ci = (int)(i - r * cin);
        const int64_t b = r / Lin;
        const int pos = (int)(r - b * Lin);
        float acc = 0.f;
        for (int tap = 0; tap < k; ++tap) {
            const int q = pos + p - tap;
            if (q < 0 || q % s) continue;
            const int o = q / s;
            if (o >= Lout) continue;
            acc += dcol[(b * Lout + o) * W + ci * k + tap];
        }
        if (ci < ca) {
            if (dxa) dxa[(b * Lin + pos) * ca + ci] += acc;
        } else if (dxb) {
            dxb[(b * Lin + pos) * cb + (ci - ca)] += acc;
        }
    }
}

// ConvTranspose1d: y(b, o, co) = bias[co] + sum over (i, tap) with i*s - p + tap = o of ycol[(b*Lin + i)][co*k + tap]
__global__ void convt_gather_kernel(int64_t B, int Lin, int Lout, int C, int k, int s, int p, const float *ycol,
                                    const float *bias, float *y)
{
    const int64_t n = B * Lout * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / C;
        const int co = (int)(i - r * C);
        const int64_t b = r / Lout;
        const int o = (int)(r - b * Lout);
        float acc = 0.f;
        for (int tap = 0; tap < k; ++tap) {
            const int q = o + p - tap;
            if (q < 0 || q % s) continue;
            const int ii = q / s;
            if (ii >= Lin) continue;
            acc += ycol[(b * Lin + ii) * (C * k) + co * k + tap];
        }
        y[i] = acc + bias[co];
    }
}

// dycol[(b*Lin + i)][co*k + tap] = dy(b, i*s - p + tap, co) (0 outside)
__global__ void convt_scatter_kernel(int64_t B, int Lin, int Lout, int C, int k, int s, int p, const float *dy,
                                     float *dycol)
{
    const int W = C * k;
    const int64_t n = B * Lin * W;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / W;
        const int j = (int)(i - r * W), co = j / k, tap = j - co * k;
        const int64_t b = r / Lin;
        const int ii = (int)(r - b * Lin), o = ii * s - p + tap;
        dycol[i] = (o >= 0 && o < Lout) ? dy[(b * Lout + o) * C + co] : 0.f;
    }
}

// GroupNorm over (L positions x C/G channels) per (row, group), eps 1e-5: one workgroup per (b, g)
__global__ __launch_bounds__(256) void gn_fwd_kernel(int L, int C, int G, const float *x, const float *w, const float *bb,
                                                     float *y, float *stat)
{
    __shared__ double s1[256], s2[256];
    const int64_t b = blockIdx.x / G;
    const int g = blockIdx.x % G, cpg = C / G, n = L * cpg;
    const float *xb = x + b * L * C + g * cpg;
    double a1 = 0, a2 = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
        const double v = xb[(i / cpg) * C + i % cpg];
        a1 += v;
        a2 += v * v;
    }
    s1[threadIdx.x] = a1;
    s2[threadIdx.x] = a2;
    __syncthreads();
    for (int m = 128; m > 0; m >>= 1) {
        if ((int)threadIdx.x < m) {
            s1[threadIdx.x] += s1[threadIdx.x + m];
            s2[threadIdx.x] += s2[threadIdx.x + m];
        }
        __syncthreads();
    }
    const double mean = s1[0] / n, var = fmax(s2[0] / n - mean * mean, 0.0);
    const float mf = (float)mean, rs = (float)(1.0 / sqrt(var + 1e-5));
    if (threadIdx.x == 0) {
        stat[2 * blockIdx.x] = mf;
        stat[2 * blockIdx.x + 1] = rs;
    }
    for (int i = threadIdx.x; i < n; i += 256) {
        const int l = i / cpg, c = g * cpg + i % cpg;
        const int64_t e = (b * L + l) * C + c;
        y[e] = (x[e] - mf) * rs * w[c] + bb[c];
    }
}

// GroupNorm backward: dx += rstd * (dxh - mean(dxh) - xh * mean(dxh * xh)), dxh = dy * w; per-row partials of
// d weight (dy * xh) and d bias (dy) into part[b][2][C] (reduced over rows by colsum afterwards)
__global__ __launch_bounds__(256) void gn_bwd_kernel(int L, int C, int G, const float *x, const float *dy, const float *w,
                                                     const float *stat, float *dx, float *part)
{
    __shared__ double s1[256], s2[256];
    const int64_t b = blockIdx.x / G;
    const int g = blockIdx.x % G, cpg = C / G, n = L * cpg;
    const float mf = stat[2 * blockIdx.x], rs = stat[2 * blockIdx.x + 1];
    double a1 = 0, a2 = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
        const int l = i / cpg, c = g * cpg + i % cpg;
        const int64_t e = (b * L + l) * C + c;
        const float xh = (x[e] - mf) * rs, d = dy[e] * w[c];
        a1 += d;
        a2 += (double)d * xh;
    }
    s1[threadIdx.x] = a1;
    s2[threadIdx.x] = a2;
    __syncthreads();
    for (int m = 128; m > 0; m >>= 1) {
        if ((int)threadIdx.x < m) {
            s1[threadIdx.x] += s1[threadIdx.x + m];
            s2[threadIdx.x] += s2[threadIdx.x + m];
        }
        __syncthreads();
    }
    const float m1 = (float)(s1[0] / n), m2 = (float)(s2[0] / n);
    for (int i = threadIdx.x; i < n; i += 256) {
        const int l = i / cpg, c = g * cpg + i % cpg;
        const int64_t e = (b * L + l) * C + c;
        const float xh = (x[e] - mf) * rs, d = dy[e] * w[c];
        dx[e] += rs * (d - m1 - xh * m2);
    }
    // affine partials: one thread per channel of the group, over the positions
    for (int cc = threadIdx.x; cc < cpg; cc += 256) {
        const int c = g * cpg + cc;
        float gw = 0.f, gb = 0.f;
        for (int l = 0; l < L; ++l) {
            const int64_t e = (b * L + l) * C + c;
            gw += dy[e] * ((x[e] - mf) * rs);
            gb += dy[e];
        }
        part[b * 2 * C + c] = gw;
        part[b * 2 * C + C + c] = gb;
    }
}

// y[b][l][c] = x[b][l][c] + cond[b][c]
__global__ void addc_kernel(int64_t B, int L, int C, const float *x, const float *cond, float *y)
{
    const int64_t n = B * L * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = x[i] + cond[(i / ((int64_t)L * C)) * C + i % C];
}

// dcond[b][c] += sum_l dy[b][l][c]
__global__ void rowsum_l_kernel(int64_t B, int L, int C, const float *dy, float *dcond)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < B * C; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / C;
        const int c = (int)(i - b * C);
        float acc = 0.f;
        for (int l = 0; l < L; ++l) acc += dy[(b * L + l) * C + c];
        dcond[i] += acc;
    }
}

__global__ void add_kernel(int64_t n, const float *a, const float *b, float *y)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = a[i] + b[i];
}

__global__ void acc_kernel(int64_t n, const float *d, float *g)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        g[i] += d[i];
}

// x_noisy = sqrt(abar_t) x0 + sqrt(1 - abar_t) noise  (q_sample, diffusion_model_base.py:421-431)
__global__ void q_sample_kernel(int64_t B, int F, const float *x0, const float *noise, const int64_t *t,
                                const float *sac, const float *s1mac, int n_steps, float *xn)
{
    const int64_t n = B * F;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t ti = min(max(t[i / F], (int64_t)0), (int64_t)n_steps - 1);  // never read past the table
        const float u = sac[ti] * x0[i], v = s1mac[ti] * noise[i];
        xn[i] = u + v;
    }
}

// SinusoidalPosEmb(32) (layers.py:249-255): [sin(t f_k), cos(t f_k)], f_k = exp(k * -(ln 1e4 / 15))
__global__ void sinemb_kernel(int64_t B, const int64_t *t, float *e)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < B * 32; i += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(i & 31), k = j & 15;
        const float f = expf((float)k * (float)(-(9.210340371976184 / 15.0)));
        const float arg = (float)t[i >> 5] * f;
        e[i] = j < 16 ? sinf(arg) : cosf(arg);
    }
}

// c_emb = cat(t_emb, ctx * (1 - mask))  (ConditionedMLPNet.forward)
__global__ void cemb_kernel(int64_t B, int T, int C, const float *temb, const float *ctx, const float *mask, float *c)
{
    const int W = T + C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < B * W; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / W;
        const int j = (int)(i - b * W);
        c[i] = j < T ? temb[b * T + j] : ctx[b * C + (j - T)] * (1.f - mask[b]);
    }
}

// loss partials: sum (o - n)^2 per block (fp64), and d out = 2 (o - n) / numel
__global__ __launch_bounds__(256) void l2_kernel(int64_t n, const float *o, const float *y, float inv_n, float *dout,
                                                 double *part)
{
    __shared__ double s[256];
    double acc = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float d = o[i] - y[i];
        acc += (double)(d * d);
        if (dout) dout[i] = (2.f * d) * inv_n;
    }
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}

// bias gradient db[n] += sum_m dy[m*ld + n]: 64 columns per workgroup, 4 row lanes, fixed order
__global__ __launch_bounds__(256) void colsum_kernel(int64_t M, int N, const float *dy, int64_t ld, float *db)
{
    __shared__ float s[4][64];
    const int c = threadIdx.x & 63, r = threadIdx.x >> 6, n = blockIdx.x * 64 + c;
    float acc = 0.f;
    if (n < N)
        for (int64_t m = r; m < M; m += 4) acc += dy[m * ld + n];
    s[r][c] = acc;
    __syncthreads();
    if (r == 0 && n < N) db[n] += (s[0][c] + s[1][c]) + (s[2][c] + s[3][c]);
}

// torch.optim.Adam single-tensor step (no weight decay, no amsgrad)
__global__ void adam_kernel(int64_t n, float *p, const float *g, float *m, float *v, float b1, float b2, float step_size,
                            float bc2_sqrt, float eps)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float gi = g[i];
        m[i] = m[i] + (1.f - b1) * (gi - m[i]);  // exp_avg.lerp_(grad, 1 - beta1)
        v[i] = v[i] * b2 + (1.f - b2) * (gi * gi);  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
        const float denom = sqrtf(v[i]) / bc2_sqrt + eps;
        p[i] = p[i] + (-step_size) * (m[i] / denom);
    }
}

__global__ void scale_kernel(int64_t n, float *g, float f)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) g[i] *= f;
}

// EMA.update_average: old * beta + (1 - beta) * new
__global__ void ema_kernel(int64_t n, float *ema, const float *p, float beta, int reset)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float old = reset ? p[i] : ema[i];
        ema[i] = old * beta + (1.f - beta) * p[i];
    }
}

unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>((n + 255) / 256, 4096); }

}  // namespace

struct Trainer {
    TrainSpec sp;
    hipStream_t st = nullptr;
    int64_t cap = 0;  // rows the activation buffers hold
    float *P = nullptr, *G = nullptr, *Mo = nullptr, *Vo = nullptr, *E = nullptr, *sched = nullptr;
    std::vector<float *> bufs;
    double *part = nullptr;
    int64_t step = 0;
    // data parallelism: every rank trains on its own rows; the flat gradient is sum-all-reduced and divided
    // by the rank count before Adam, so the ranks' parameters stay identical (DistributedDataParallel's rule)
    Comm *comm = nullptr;
    std::string comm_err;

    ~Trainer()
    {
        for (float *b : bufs) (void)hipFree(b);
        for (float *b : {P, G, Mo, Vo, E, sched, ws}) (void)hipFree(b);
        (void)hipFree(part);
        delete comm;
    }
    float *alloc(int64_t n)
    {
        float *p = nullptr;
        if (hipMalloc(&p, (size_t)std::max<int64_t>(n, 1) * 4) != hipSuccess) return nullptr;
        bufs.push_back(p);
        return p;
    }
    // split-K / split-row workspace (grown on demand; the stream orders its reuse)
    float *ws = nullptr;
    int64_t ws_n = 0;
    float *workspace(int64_t n)
    {
        if (n > ws_n) {
            (void)hipStreamSynchronize(st);
            (void)hipFree(ws);
            ws = nullptr;
            ws_n = 0;
            if (hipMalloc(&ws, (size_t)n * 4) != hipSuccess) return nullptr;
            ws_n = n;
        }
        return ws;
    }
    // the fp32 MFMA GEMM (default) or the VALU one (MPCD_TRAIN_GEMM=valu)
    static decltype(&gemm_kernel) gemm_fn()
    {
        static const bool valu = [] {
            const char *e = getenv("MPCD_TRAIN_GEMM");
            return e && !strcmp(e, "valu");
        }();
        return valu ? &gemm_kernel : &gemm_mfma_kernel;
    }
    hipError_t gemm(int M, int N, int K, const float *a, int64_t sam, int64_t sak, const float *b, int64_t sbk,
                    int64_t sbn, float *c, int64_t ldc, float beta, const float *bias, float *db = nullptr)
    {
        dim3 g((N + GT - 1) / GT, (M + GT - 1) / GT);
        const int64_t tiles = (int64_t)g.x * g.y;
        // the weight-gradient GEMMs (M, N <= a few hundred, K = rows) would occupy a handful of CUs: split K
        int z = 1;
        if (tiles < 256 && K >= 512) z = (int)std::min<int64_t>(std::max<int64_t>(512 / tiles, 1), K / 256);
        // db (optional): db[m] += sum_k A(m,k), taken from the staged A tiles (slices reduced in z order)
        if (z > 1) {
            const int kchunk = ((K + z - 1) / z + GK - 1) / GK * GK;
            z = (K + kchunk - 1) / kchunk;
            const int64_t mn = (int64_t)M * N;
            float *part = workspace(mn * z + (db ? (int64_t)M * z : 0));
            if (!part) return hipErrorOutOfMemory;
            float *rs = db ? part + mn * z : nullptr;
            g.z = z;
            hipLaunchKernelGGL(gemm_fn(), g, dim3(256), 0, st, M, N, K, a, sam, sak, b, sbk, sbn, part, (int64_t)N, 0.f,
                               (const float *)nullptr, kchunk, mn, rs);
            hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid_for(mn)), dim3(256), 0, st, M, N, z, (const float *)part, c,
                               ldc, beta, bias);
            if (db)
                hipLaunchKernelGGL(colsum_reduce_kernel, dim3((M + 255) / 256), dim3(256), 0, st, M, z, (const float *)rs,
                                   db);
            return hipGetLastError();
        }
        float *rs = nullptr;
        if (db && !(rs = workspace(M))) return hipErrorOutOfMemory;
        hipLaunchKernelGGL(gemm_fn(), g, dim3(256), 0, st, M, N, K, a, sam, sak, b, sbk, sbn, c, ldc, beta, bias, K,
                           (int64_t)0, rs);
        if (db) hipLaunchKernelGGL(colsum_reduce_kernel, dim3((M + 255) / 256), dim3(256), 0, st, M, 1, (const float *)rs, db);
        return hipGetLastError();
    }
    // db[n] += sum_m dy[m*ld + n], rows split over workgroups, slices reduced in order
    hipError_t colsum(int64_t M, int N, const float *dy, int64_t ld, float *db)
    {
        const int64_t rchunk = 256;
        const int z = (int)std::min<int64_t>((M + rchunk - 1) / rchunk, 65535);
        const int64_t rc = (M + z - 1) / z;
        float *part = workspace((int64_t)z * N);
        if (!part) return hipErrorOutOfMemory;
        hipLaunchKernelGGL(colsum_part_kernel, dim3((N + 63) / 64, z), dim3(256), 0, st, M, N, dy, ld, rc, part);
        hipLaunchKernelGGL(colsum_reduce_kernel, dim3((N + 255) / 256), dim3(256), 0, st, N, z, (const float *)part, db);
        return hipGetLastError();
    }
    // Y[B][N] = X[B][K] W[N][K]^T + b   (X rows of stride ldx; W rows of stride ldw, starting at column koff)
    hipError_t lin(int64_t B, const float *x, int ldx, const TrainLin &L, int koff, int K, float *y, float beta, bool bias)
    {
        return gemm((int)B, L.n, K, x, ldx, 1, P + L.w + koff, 1, L.k, y, L.n, beta, bias ? P + L.b : nullptr);
    }
    // backward of Y = X W[:, koff:koff+K]^T: dW[:, koff..] += dY^T X; dX (+)= dY W[:, koff..];
    // with_bias: db += column sums of dY, folded into the dW GEMM's staged dY tiles
    hipError_t lin_bwd(int64_t B, const float *x, int ldx, const TrainLin &L, int koff, int K, const float *dy, float *dx,
                       float dx_beta, bool with_bias = false)
    {
        hipError_t e = gemm(L.n, K, (int)B, dy, 1, L.n, x, ldx, 1, G + L.w + koff, L.k, 1.f, nullptr,
                            with_bias ? G + L.b : nullptr);
        if (e == hipSuccess && dx) e = gemm((int)B, K, L.n, dy, L.n, 1, P + L.w + koff, L.k, 1, dx, K, dx_beta, nullptr);
        return e;
    }
    void mish(int64_t n, const float *pre, float *out)
    {
        hipLaunchKernelGGL(mish_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, pre, out);
    }
    void mish_bwd(int64_t n, const float *pre, const float *dout, float *dpre, int acc = 0)
    {
        hipLaunchKernelGGL(mish_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, pre, dout, dpre, acc);
    }

    // ---- U-Net trunk tape: per tensor value / gradient, per op scratch (im2col, GroupNorm statistics)
    struct UBuf {
        float *v = nullptr, *g = nullptr;
    };
    std::vector<UBuf> U;
    std::vector<float *> ucol, ustat, upart;
    float *ugrad = nullptr;  // every trunk gradient buffer in one slab: one memset per step
    int64_t ugrad_n = 0;
    int tL(int t) const { return sp.ut[t].L; }
    int tC(int t) const { return sp.ut[t].C; }

    int reserve_unet(int64_t B)
    {
        const int nt = (int)sp.ut.size(), no = (int)sp.uops.size();
        U.assign(nt, UBuf{});
        U[UT_XNOISY] = {A.xn, nullptr};
        U[UT_MC] = {A.mc, A.dmc};
        std::vector<int64_t> goff(nt, 0);
        ugrad_n = 0;
        for (int t = 2; t < nt; ++t) {
            if (t == sp.u_out) continue;
            goff[t] = ugrad_n;
            ugrad_n += (B * tL(t) * tC(t) + 63) / 64 * 64;
        }
        if (!(ugrad = alloc(ugrad_n))) return -1;
        for (int t = 2; t < nt; ++t) {
            if (t == sp.u_out) {
                U[t] = {A.out, A.dout};
                continue;
            }
            U[t].v = alloc(B * tL(t) * tC(t));
            U[t].g = ugrad + goff[t];
        }
        ucol.assign(no, nullptr);
        ustat = upart = ucol;
        for (int i = 0; i < no; ++i) {
            const UOp &o = sp.uops[i];
            if (o.kind == UOP_CONV) {
                const int cin = tC(o.in0) + (o.in1 >= 0 ? tC(o.in1) : 0);
                ucol[i] = alloc(B * tL(o.out) * cin * o.k);
            } else if (o.kind == UOP_CONVT) {
                ucol[i] = alloc(B * tL(o.in0) * tC(o.out) * o.k);
            } else if (o.kind == UOP_GN) {
                ustat[i] = alloc(2 * B * o.groups);
                upart[i] = alloc(2 * B * tC(o.out));
            }
        }
        return 0;
    }

    hipError_t unet_fwd(int64_t B)
    {
        hipError_t e = hipSuccess;
        for (size_t i = 0; i < sp.uops.size() && e == hipSuccess; ++i) {
            const UOp &o = sp.uops[i];
            const float *x0 = U[o.in0].v, *x1 = o.in1 >= 0 ? U[o.in1].v : nullptr;
            float *y = U[o.out].v;
            const int Li = tL(o.in0), Lo = tL(o.out), Ci = tC(o.in0), Co = tC(o.out);
            switch (o.kind) {
            case UOP_CONV: {
                const int cb = o.in1 >= 0 ? tC(o.in1) : 0, K = (Ci + cb) * o.k;
                hipLaunchKernelGGL(im2col_kernel, dim3(grid_for(B * Lo * K)), dim3(256), 0, st, B, Li, Lo, Ci, cb, o.k,
                                   o.s, o.p, x0, x1, ucol[i]);
                e = gemm((int)(B * Lo), Co, K, ucol[i], K, 1, P + o.w, 1, K, y, Co, 0.f, P + o.b);
                break;
            }
            case UOP_CONVT: {
                const int K = Co * o.k;
                e = gemm((int)(B * Li), K, Ci, x0, Ci, 1, P + o.w, K, 1, ucol[i], K, 0.f, nullptr);
                hipLaunchKernelGGL(convt_gather_kernel, dim3(grid_for(B * Lo * Co)), dim3(256), 0, st, B, Li, Lo, Co,
                                   o.k, o.s, o.p, ucol[i], P + o.b, y);
                break;
            }
            case UOP_GN:
                hipLaunchKernelGGL(gn_fwd_kernel, dim3((unsigned)(B * o.groups)), dim3(256), 0, st, Li, Ci, o.groups, x0,
                                   P + o.w, P + o.b, y, ustat[i]);
                break;
            case UOP_MISH: mish(B * Li * Ci, x0, y); break;
            case UOP_ADDC:
                hipLaunchKernelGGL(addc_kernel, dim3(grid_for(B * Li * Ci)), dim3(256), 0, st, B, Li, Ci, x0, x1, y);
                break;
            case UOP_ADD:
                hipLaunchKernelGGL(add_kernel, dim3(grid_for(B * Li * Ci)), dim3(256), 0, st, B * Li * Ci, x0, x1, y);
                break;
            case UOP_LIN: e = gemm((int)(B * Li), Co, Ci, x0, Ci, 1, P + o.w, 1, Ci, y, Co, 0.f, P + o.b); break;
            }
            if (e == hipSuccess) e = hipGetLastError();
        }
        return e;
    }

    hipError_t unet_bwd(int64_t B)
    {
        hipError_t e = hipSuccess;
        for (int i = (int)sp.uops.size() - 1; i >= 0 && e == hipSuccess; --i) {
            const UOp &o = sp.uops[i];
            const float *x0 = U[o.in0].v, *go = U[o.out].g;
            float *g0 = U[o.in0].g, *g1 = o.in1 >= 0 ? U[o.in1].g : nullptr;
            const int Li = tL(o.in0), Lo = tL(o.out), Ci = tC(o.in0), Co = tC(o.out);
            switch (o.kind) {
            case UOP_CONV: {
                const int cb = o.in1 >= 0 ? tC(o.in1) : 0, K = (Ci + cb) * o.k;
                const int64_t R = B * Lo;
                e = gemm(Co, K, (int)R, go, 1, Co, ucol[i], K, 1, G + o.w, K, 1.f, nullptr, G + o.b);
                if (e == hipSuccess && (g0 || g1)) {
                    e = gemm((int)R, K, Co, go, Co, 1, P + o.w, K, 1, ucol[i], K, 0.f, nullptr);
                    hipLaunchKernelGGL(col2im_kernel, dim3(grid_for(B * Li * (Ci + cb))), dim3(256), 0, st, B, Li, Lo, Ci,
                                       cb, o.k, o.s, o.p, ucol[i], g0, g1);
                }
                break;
            }
            case UOP_CONVT: {
                const int K = Co * o.k;
                hipLaunchKernelGGL(convt_scatter_kernel, dim3(grid_for(B * Li * K)), dim3(256), 0, st, B, Li, Lo, Co, o.k,
                                   o.s, o.p, go, ucol[i]);
                e = gemm(Ci, K, (int)(B * Li), x0, 1, Ci, ucol[i], K, 1, G + o.w, K, 1.f, nullptr);
                if (e == hipSuccess) e = colsum(B * Lo, Co, go, (int64_t)Co, G + o.b);
                if (e == hipSuccess && g0) e = gemm((int)(B * Li), Ci, K, ucol[i], K, 1, P + o.w, 1, K, g0, Ci, 1.f, nullptr);
                break;
            }
            case UOP_GN:
                hipLaunchKernelGGL(gn_bwd_kernel, dim3((unsigned)(B * o.groups)), dim3(256), 0, st, Li, Ci, o.groups, x0, go,
                                   P + o.w, ustat[i], g0, upart[i]);
                if (o.b == o.w + Ci) {  // weight and bias adjacent in the flat buffer: one pass over [B][2C]
                    e = colsum(B, 2 * Ci, upart[i], (int64_t)2 * Ci, G + o.w);
                } else {
                    e = colsum(B, Ci, upart[i], (int64_t)2 * Ci, G + o.w);
                    if (e == hipSuccess) e = colsum(B, Ci, upart[i] + Ci, (int64_t)2 * Ci, G + o.b);
                }
                break;
            case UOP_MISH: mish_bwd(B * Li * Ci, x0, go, g0, 1); break;
            case UOP_ADDC:
                hipLaunchKernelGGL(acc_kernel, dim3(grid_for(B * Li * Ci)), dim3(256), 0, st, B * Li * Ci, go, g0);
                hipLaunchKernelGGL(rowsum_l_kernel, dim3(grid_for(B * Ci)), dim3(256), 0, st, B, Li, Ci, go, g1);
                break;
            case UOP_ADD:
                hipLaunchKernelGGL(acc_kernel, dim3(grid_for(B * Li * Ci)), dim3(256), 0, st, B * Li * Ci, go, g0);
                hipLaunchKernelGGL(acc_kernel, dim3(grid_for(B * Li * Ci)), dim3(256), 0, st, B * Li * Ci, go, g1);
                break;
            case UOP_LIN: {
                const int64_t R = B * Li;
                e = gemm(Co, Ci, (int)R, go, 1, Co, x0, Ci, 1, G + o.w, Ci, 1.f, nullptr, G + o.b);
                if (e == hipSuccess && g0) e = gemm((int)R, Ci, Co, go, Co, 1, P + o.w, Ci, 1, g0, Ci, 1.f, nullptr);
                break;
            }
            }
            if (e == hipSuccess) e = hipGetLastError();
        }
        return e;
    }

    // activation buffers per training row count
    struct Act {
        float *xn, *e, *p1, *q1, *temb, *cemb, *mc, *f1, *out, *dout, *dmc, *dcemb, *dq1, *tmp;
        std::vector<float *> a1, h1, s, y, dy, dh;  // per block
    } A{};

    int reserve(int64_t B)
    {
        if (B <= cap) return 0;
        for (float *b : bufs) (void)hipFree(b);
        bufs.clear();
        const int F = sp.flat, T = sp.temb, W = sp.temb + sp.ctx_dim, nb = (int)sp.blocks.size();
        A.xn = alloc(B * F);
        A.e = alloc(B * 32);
        A.p1 = alloc(B * 128);
        A.q1 = alloc(B * 128);
        A.temb = alloc(B * T);
        A.cemb = alloc(B * W);
        A.mc = alloc(B * W);
        A.f1 = alloc(B * sp.base);
        A.out = alloc(B * F);
        A.dout = alloc(B * F);
        A.dmc = alloc(B * W);
        A.dcemb = alloc(B * W);
        A.dq1 = alloc(B * 128);
        int wtmp = std::max(256, sp.base);  // widest backward scratch: d(h1) / d(a1) of every block, d(f1)
        for (int j = 0; j < nb; ++j) wtmp = std::max(wtmp, sp.blocks[j].co);
        A.tmp = alloc(B * wtmp);
        A.a1.assign(nb, nullptr);
        A.h1 = A.s = A.y = A.dy = A.dh = A.a1;
        for (int j = 0; j < nb; ++j) {
            const int co = sp.blocks[j].co;
            A.a1[j] = alloc(B * co);
            A.h1[j] = alloc(B * co);
            A.s[j] = alloc(B * co);
            A.y[j] = alloc(B * co);
            A.dy[j] = alloc(B * co);
            A.dh[j] = alloc(B * co);
        }
        if (sp.unet && reserve_unet(B) != 0) return -1;
        for (float *b : bufs)
            if (!b) return -1;
        cap = B;
        return 0;
    }

    // block j's input: x_noisy (first down), the previous block's output, or the concat (y_prev, skip)
    hipError_t block_fwd(int64_t B, int j)
    {
        const TrainBlock &k = sp.blocks[j];
        hipError_t e;
        const float *x0 = k.in0 < 0 ? A.xn : A.y[k.in0];
        const int c0 = k.in0 < 0 ? sp.flat : sp.blocks[k.in0].co;
        e = lin(B, x0, c0, k.la, 0, c0, A.a1[j], 0.f, true);
        if (e == hipSuccess && k.in1 >= 0) e = lin(B, A.y[k.in1], sp.blocks[k.in1].co, k.la, c0, sp.blocks[k.in1].co, A.a1[j], 1.f, false);
        if (e != hipSuccess) return e;
        mish(B * k.co, A.a1[j], A.h1[j]);
        e = lin(B, A.h1[j], k.co, k.lb, 0, k.co, A.s[j], 0.f, true);
        if (e == hipSuccess) e = lin(B, A.mc, sp.temb + sp.ctx_dim, k.lc, 0, sp.temb + sp.ctx_dim, A.s[j], 1.f, true);
        if (e != hipSuccess) return e;
        mish(B * k.co, A.s[j], A.y[j]);
        return hipGetLastError();
    }
    // given dy[j] (gradient of block j's output), accumulate parameter grads, dmc, and the inputs' grads
    hipError_t block_bwd(int64_t B, int j)
    {
        const TrainBlock &k = sp.blocks[j];
        const int W = sp.temb + sp.ctx_dim;
        hipError_t e;
        mish_bwd(B * k.co, A.s[j], A.dy[j], A.dh[j]);  // d s
        e = lin_bwd(B, A.mc, W, k.lc, 0, W, A.dh[j], A.dmc, 1.f, true);
        if (e == hipSuccess) e = lin_bwd(B, A.h1[j], k.co, k.lb, 0, k.co, A.dh[j], A.tmp, 0.f, true);  // d h1 -> tmp
        if (e != hipSuccess) return e;
        mish_bwd(B * k.co, A.a1[j], A.tmp, A.tmp);  // d a1
        const float *x0 = k.in0 < 0 ? A.xn : A.y[k.in0];
        const int c0 = k.in0 < 0 ? sp.flat : sp.blocks[k.in0].co;
        e = lin_bwd(B, x0, c0, k.la, 0, c0, A.tmp, k.in0 < 0 ? nullptr : A.dy[k.in0], 1.f, true);
        if (e == hipSuccess && k.in1 >= 0)
            e = lin_bwd(B, A.y[k.in1], sp.blocks[k.in1].co, k.la, c0, sp.blocks[k.in1].co, A.tmp, A.dy[k.in1], 1.f);
        return e;
    }

    hipError_t run(int64_t B, const float *x0, const float *ctx, const int64_t *t, const float *noise, const float *mask,
                   bool update, double *loss)
    {
        const int F = sp.flat, T = sp.temb, C = sp.ctx_dim, W = T + C;
        const int nb = (int)sp.blocks.size();
        hipError_t e;
        // ---- forward (p_losses)
        hipLaunchKernelGGL(q_sample_kernel, dim3(grid_for(B * F)), dim3(256), 0, st, B, F, x0, noise, t, sched,
                           sched + sp.n_steps, sp.n_steps, A.xn);
        hipLaunchKernelGGL(sinemb_kernel, dim3(grid_for(B * 32)), dim3(256), 0, st, B, t, A.e);
        if ((e = lin(B, A.e, 32, sp.t1, 0, 32, A.p1, 0.f, true)) != hipSuccess) return e;
        mish(B * 128, A.p1, A.q1);
        if ((e = lin(B, A.q1, 128, sp.t2, 0, 128, A.temb, 0.f, true)) != hipSuccess) return e;
        hipLaunchKernelGGL(cemb_kernel, dim3(grid_for(B * W)), dim3(256), 0, st, B, T, C, A.temb, ctx, mask, A.cemb);
        mish(B * W, A.cemb, A.mc);
        const int last = nb - 1;
        if (sp.unet) {
            if ((e = unet_fwd(B)) != hipSuccess) return e;
        } else {
            for (int j = 0; j < nb; ++j)
                if ((e = block_fwd(B, j)) != hipSuccess) return e;
            if ((e = lin(B, A.y[last], sp.base, sp.f1, 0, sp.base, A.f1, 0.f, true)) != hipSuccess) return e;
            if ((e = lin(B, A.f1, sp.base, sp.f2, 0, sp.base, A.out, 0.f, true)) != hipSuccess) return e;
        }
        // ---- loss = mean((eps - noise)^2)  (WeightedL2, predict_epsilon)
        const int64_t n = B * F;
        const unsigned nbk = std::min<unsigned>(grid_for(n), 1024);
        hipLaunchKernelGGL(l2_kernel, dim3(nbk), dim3(256), 0, st, n, A.out, noise, (float)(1.0 / (double)n),
                           update ? A.dout : nullptr, part);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        std::vector<double> hp(nbk);
        if ((e = hipMemcpyAsync(hp.data(), part, nbk * sizeof(double), hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if (!update) {
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
            double s = 0;
            for (double v : hp) s += v;
            *loss = s / (double)n;
            return hipSuccess;
        }
        // ---- backward
        if ((e = hipMemsetAsync(G, 0, (size_t)sp.n_params * 4, st)) != hipSuccess) return e;
        for (int j = 0; j < nb; ++j)
            if ((e = hipMemsetAsync(A.dy[j], 0, (size_t)B * sp.blocks[j].co * 4, st)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(A.dmc, 0, (size_t)B * W * 4, st)) != hipSuccess) return e;
        if (sp.unet) {
            if ((e = hipMemsetAsync(ugrad, 0, (size_t)ugrad_n * 4, st)) != hipSuccess) return e;
            if ((e = unet_bwd(B)) != hipSuccess) return e;
        } else {
            if ((e = lin_bwd(B, A.f1, sp.base, sp.f2, 0, sp.base, A.dout, A.tmp, 0.f, true)) != hipSuccess) return e;  // d f1
            if ((e = lin_bwd(B, A.y[last], sp.base, sp.f1, 0, sp.base, A.tmp, A.dy[last], 1.f, true)) != hipSuccess)
                return e;
            for (int j = nb - 1; j >= 0; --j)
                if ((e = block_bwd(B, j)) != hipSuccess) return e;
        }
        mish_bwd(B * W, A.cemb, A.dmc, A.dcemb);
        // time MLP: d t_emb = d c_emb[:, :T] (row stride W)
        if ((e = gemm(sp.t2.n, 128, (int)B, A.dcemb, 1, W, A.q1, 128, 1, G + sp.t2.w, 128, 1.f, nullptr, G + sp.t2.b)) !=
            hipSuccess)
            return e;
        if ((e = gemm((int)B, 128, T, A.dcemb, W, 1, P + sp.t2.w, 128, 1, A.dq1, 128, 0.f, nullptr)) != hipSuccess) return e;
        mish_bwd(B * 128, A.p1, A.dq1, A.dq1);
        if ((e = lin_bwd(B, A.e, 32, sp.t1, 0, 32, A.dq1, nullptr, 0.f, true)) != hipSuccess) return e;
        // ---- data-parallel gradient average: one all-reduce of the whole flat gradient (a single bucket:
        // 0.6 MB for the cfg2 MLP, 4 MB for the cart-pole U-Net, tens of microseconds over xGMI)
        if (comm && comm->nranks > 1) {
            if (comm->allreduce(G, (size_t)sp.n_params, COMM_SUM_F32, st, comm_err) != 0) return hipErrorUnknown;
            hipLaunchKernelGGL(scale_kernel, dim3(grid_for(sp.n_params)), dim3(256), 0, st, (int64_t)sp.n_params, G,
                               1.f / (float)comm->nranks);
        }
        // ---- Adam, then the EMA model (trainer.py: optimizer step, then every update_ema_every steps)
        ++step;
        const double bc1 = 1.0 - std::pow((double)sp.beta1, (double)step), bc2 = 1.0 - std::pow((double)sp.beta2, (double)step);
        hipLaunchKernelGGL(adam_kernel, dim3(grid_for(sp.n_params)), dim3(256), 0, st, (int64_t)sp.n_params, P, G, Mo, Vo,
                           sp.beta1, sp.beta2, (float)(sp.lr / bc1), (float)std::sqrt(bc2), sp.eps);
        const int64_t s0 = step - 1;  // trainer's train_steps_current before its increment
        if (sp.update_ema_every > 0 && s0 % sp.update_ema_every == 0)
            hipLaunchKernelGGL(ema_kernel, dim3(grid_for(sp.n_params)), dim3(256), 0, st, (int64_t)sp.n_params, E, P,
                               sp.ema_decay, s0 < sp.step_start_ema ? 1 : 0);
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        double s = 0;
        for (double v : hp) s += v;
        *loss = s / (double)n;
        return hipGetLastError();
    }
};

Trainer *trainer_new(const TrainSpec &sp, const float *params_host, const float *sched_host, std::string *why)
{
    Trainer *t = new Trainer;
    t->sp = sp;
    const size_t pb = (size_t)sp.n_params * 4;
    bool ok = hipMalloc(&t->P, pb) == hipSuccess && hipMalloc(&t->G, pb) == hipSuccess &&
              hipMalloc(&t->Mo, pb) == hipSuccess && hipMalloc(&t->Vo, pb) == hipSuccess &&
              hipMalloc(&t->E, pb) == hipSuccess && hipMalloc(&t->sched, (size_t)sp.n_steps * 2 * 4) == hipSuccess &&
              hipMalloc(&t->part, 1024 * sizeof(double)) == hipSuccess;
    ok = ok && hipMemcpy(t->P, params_host, pb, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(t->E, params_host, pb, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemset(t->Mo, 0, pb) == hipSuccess && hipMemset(t->Vo, 0, pb) == hipSuccess &&
         hipMemset(t->G, 0, pb) == hipSuccess &&
         hipMemcpy(t->sched, sched_host, (size_t)sp.n_steps * 2 * 4, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) {
        if (why) *why = "trainer: device allocation / upload failed";
        delete t;
        return nullptr;
    }
    return t;
}

int trainer_step(Trainer *t, const TrainBatch &b, bool update, double *loss, std::string *why)
{
    t->st = (hipStream_t)b.stream;
    t->comm_err.clear();  // a previous step's all-reduce failure must not label this step's errors
    if (t->reserve(b.batch) != 0) {
        if (why) *why = "trainer: activation buffers";
        return -1;
    }
    const hipError_t e = t->run(b.batch, b.x0, b.ctx, b.t, b.noise, b.mask, update, loss);
    if (e != hipSuccess) {
        if (why) *why = !t->comm_err.empty() ? "trainer: gradient all-reduce: " + t->comm_err
                                             : std::string("trainer: ") + hipGetErrorString(e);
        return -2;
    }
    return 0;
}

int trainer_set_comm(Trainer *t, Comm *c)
{
    if (t->comm) return -1;
    t->comm = c;
    return 0;
}

int trainer_read(Trainer *t, int which, float *host, size_t n)
{
    if (n != (size_t)t->sp.n_params) return -1;
    const float *src = which == 0 ? t->P : which == 1 ? t->E : which == 2 ? t->G : which == 3 ? t->Mo : t->Vo;
    return hipMemcpy(host, src, n * 4, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}

int64_t trainer_steps(Trainer *t) { return t->step; }

void trainer_free(Trainer *t) { delete t; }
