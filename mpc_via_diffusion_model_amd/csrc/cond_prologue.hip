// Timestep embedding + conditioning projections.
//
// Reference, per denoise step and per forward (x2 for CFG), per candidate:
//   t_emb = TimeEncoder(t)        SinusoidalPosEmb(32) -> Linear(32,128) -> Mish -> Linear(128,32)
//                                 (layers.py:229-255)
//   c_emb = cat(t_emb, ctx*(1-mask)).float()                      (temporal_unet.py:296-314)
//   cond_j = Linear_j(Mish(c_emb))  for every residual / MLP block (layers.py:334-338, 368-372)
// t_emb depends only on t and ctx only on the candidate, and Linear_j(Mish(cat(a, b))) =
// W_j[:, :T].Mish(a) + b_j + W_j[:, T:].Mish(b) exactly (Mish is elementwise; the masked branch's
// Mish(0) = 0 terms vanish). So the cond bias of every block is tproj[step] (+ cproj[candidate]
// for the unmasked branch), computed here once per sample call instead of 2 x S x B times.
#include <hip/hip_runtime.h>

#include "internal.h"

namespace {

constexpr int TDIM = 32;    // SinusoidalPosEmb / time_emb_dim
static_assert(TDIM == kCondTdim, "ctx_proj_col's time columns");
constexpr int THID = 128;   // TimeEncoder hidden = 4 * 32

__global__ __launch_bounds__(128) void time_prologue_kernel(const StepPlan *plan, const float *w1, const float *b1,
                                                            const float *w2, const float *b2, const CondLayer *layers,
                                                            int n_layers, int cond_dim, int cond_total, float *tproj)
{
    __shared__ float emb[TDIM], hid[THID], mt[TDIM];
    const int s = blockIdx.x, tid = threadIdx.x;
    const float t = (float)plan[s].t;
    if (tid < TDIM) {
        // emb = exp(arange(16) * -(log(10000)/15)); [sin(t*emb), cos(t*emb)] in fp32 (layers.py:249-255)
        const int k = tid & 15;
        const float neg = (float)(-(9.210340371976184 / 15.0));
        const float f = expf((float)k * neg);
        const float arg = t * f;
        emb[tid] = tid < 16 ? sinf(arg) : cosf(arg);
    }
    __syncthreads();
    // dot products accumulate in fp64 and round once: this tiny per-step prologue then carries
    // less error than the reference's own fp32 GEMMs
    {
        double acc = 0.0;
        for (int k = 0; k < TDIM; ++k) acc += (double)w1[tid * TDIM + k] * (double)emb[k];
        hid[tid] = mish_precise((float)(acc + (double)b1[tid]));
    }
    __syncthreads();
    if (tid < TDIM) {
        double acc = 0.0;
        for (int k = 0; k < THID; ++k) acc += (double)w2[tid * THID + k] * (double)hid[k];
        mt[tid] = mish_precise((float)(acc + (double)b2[tid]));  // cond_mlp's leading Mish on the time part of c_emb
    }
    __syncthreads();
    for (int l = 0; l < n_layers; ++l) {
        const CondLayer L = layers[l];
        for (int n = tid; n < L.width; n += blockDim.x) {
            double acc = 0.0;
            for (int k = 0; k < TDIM; ++k) acc += (double)L.W[(size_t)n * cond_dim + k] * (double)mt[k];
            tproj[(size_t)s * cond_total + L.off + n] = (float)(acc + (double)L.b[n]);
        }
    }
}

__global__ __launch_bounds__(256) void ctx_prologue_kernel(const float *ctx, int64_t n_rows, int ctx_dim,
                                                           const CondLayer *layers, int n_layers, int cond_dim,
                                                           int cond_total, float *cproj)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_rows * cond_total) return;
    const int64_t row = i / cond_total;
    const int col = (int)(i - row * cond_total);
    int l = 0;
    while (l + 1 < n_layers && layers[l + 1].off <= col) ++l;
    const CondLayer L = layers[l];
    const int n = col - L.off;
    double acc = 0.0;
    for (int k = 0; k < ctx_dim; ++k) acc += (double)L.W[(size_t)n * cond_dim + TDIM + k] * (double)mish_precise(ctx[row * ctx_dim + k]);
    cproj[i] = (float)acc;
}

// ctx_prologue_kernel for one shared row given by value
__global__ __launch_bounds__(256) void ctx_prologue_row_kernel(const CtxRowArg row, int ctx_dim, const CondLayer *layers,
                                                               int n_layers, int cond_dim, int cond_total, float *cproj)
{
    const int col = blockIdx.x * blockDim.x + threadIdx.x;
    if (col >= cond_total) return;
    cproj[col] = ctx_proj_col(row, ctx_dim, layers, n_layers, cond_dim, col);
}

}  // namespace

void launch_ctx_prologue_row(const CtxRowArg &row, int ctx_dim, const CondLayer *layers_dev, int n_layers,
                             int cond_dim, int cond_total, float *cproj, hipStream_t stream)
{
    hipLaunchKernelGGL(ctx_prologue_row_kernel, dim3((unsigned)((cond_total + 255) / 256)), dim3(256), 0, stream, row,
                       ctx_dim, layers_dev, n_layers, cond_dim, cond_total, cproj);
}

void launch_time_prologue(const StepPlan *plan, int n_steps, const float *time_w1, const float *time_b1,
                          const float *time_w2, const float *time_b2, const CondLayer *layers_dev, int n_layers,
                          int cond_dim, int cond_total, float *tproj, hipStream_t stream)
{
    hipLaunchKernelGGL(time_prologue_kernel, dim3(n_steps), dim3(128), 0, stream, plan, time_w1, time_b1, time_w2,
                       time_b2, layers_dev, n_layers, cond_dim, cond_total, tproj);
}

void launch_ctx_prologue(const float *ctx, int64_t n_rows, int ctx_dim, const CondLayer *layers_dev, int n_layers,
                         int cond_dim, int cond_total, float *cproj, hipStream_t stream)
{
    const int64_t n = n_rows * cond_total;
    hipLaunchKernelGGL(ctx_prologue_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, ctx, n_rows,
                       ctx_dim, layers_dev, n_layers, cond_dim, cond_total, cproj);
}

// The samplers' in-kernel noise for candidates [goff, goff + n): out[k][b][4q..4q+3] =
// philox_normal4(seed, goff + b, k, q) - the same call the MLP / U-Net kernels make for slice k.
__global__ void philox_noise_kernel(uint64_t seed, int64_t goff, int64_t n, int n_slices, int quads, float *out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = n * quads;
    if (i >= per * n_slices) return;
    const int k = (int)(i / per);
    const int64_t r = i - (int64_t)k * per;
    const int64_t b = r / quads;
    const int q = (int)(r - b * quads);
    *reinterpret_cast<f32x4 *>(out + 4 * i) = philox_normal4(seed, (uint64_t)(goff + b), (uint32_t)k, (uint32_t)q);
}

hipError_t launch_philox_noise(uint64_t seed, int64_t goff, int64_t n, int n_slices, int flat, float *out,
                               hipStream_t stream)
{
    const int64_t total = n * (flat / 4) * n_slices;
    const int64_t blocks = (total + 255) / 256;
    if (blocks > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(philox_noise_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, seed, goff, n, n_slices,
                       flat / 4, out);
    return hipGetLastError();
}
