// Internal (non-ABI) declarations shared by the libmpcd.so translation units.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "../../include/mpcd.h"
#include "common.h"

// One conditioning Linear (cond_mlp.1 of a residual / MLP block): out width `width`, weight
// [width][cond_dim] row-major, written at column `off` of the per-step / per-candidate tables.
struct CondLayer {
    const float *W;
    const float *b;
    int32_t width;
    int32_t off;
};

// Time-embedding prologue: tproj[s][off_j + n] = cond_mlp_j.W[n, :T] . Mish(t_emb(t_s)) + b_j[n]
void launch_time_prologue(const StepPlan *plan, int n_steps, const float *time_w1, const float *time_b1,
                          const float *time_w2, const float *time_b2, const CondLayer *layers_dev, int n_layers,
                          int cond_dim, int cond_total, float *tproj, hipStream_t stream);

// Context prologue: cproj[b][off_j + n] = cond_mlp_j.W[n, T:] . Mish(ctx_b)   (no bias)
void launch_ctx_prologue(const float *ctx, int64_t n_rows, int ctx_dim, const CondLayer *layers_dev, int n_layers,
                         int cond_dim, int cond_total, float *cproj, hipStream_t stream);
// one shared context row passed by value (mpcd_mpc_step: no host-to-device copy before the sampler)
constexpr int kCtxRowMax = 64;
struct CtxRowArg {
    float v[kCtxRowMax];
};
constexpr int kCondTdim = 32;  // time_emb_dim: the cond Linears' first input columns (cond_prologue.hip TDIM)
// Column col of one shared context row's projection, cond_mlp_j.W[n, T:] . Mish(ctx) in fp64: the body of
// ctx_prologue_row_kernel, and of the fp16 MLP kernel's in-launch form (mpcd_mpc_step), so both give the same bits
MPCD_DEV float ctx_proj_col(const CtxRowArg &row, int ctx_dim, const CondLayer *layers, int n_layers, int cond_dim,
                            int col)
{
    int l = 0;
    while (l + 1 < n_layers && layers[l + 1].off <= col) ++l;
    const CondLayer L = layers[l];
    const int n = col - L.off;
    double acc = 0.0;
    for (int k = 0; k < ctx_dim; ++k)
        acc += (double)L.W[(size_t)n * cond_dim + kCondTdim + k] * (double)mish_precise(row.v[k]);
    return (float)acc;
}
void launch_ctx_prologue_row(const CtxRowArg &row, int ctx_dim, const CondLayer *layers_dev, int n_layers,
                             int cond_dim, int cond_total, float *cproj, hipStream_t stream);

// The samplers' Philox noise stream for candidates [goff, goff + n): out [n_slices][n][flat] (mpcd_philox_noise)
hipError_t launch_philox_noise(uint64_t seed, int64_t goff, int64_t n, int n_slices, int flat, float *out,
                               hipStream_t stream);

// Thread-safe launch state (several host threads may launch, e.g. the loopback communicator's ranks):
// allow_max_lds<&kernel>() raises the kernel's dynamic-LDS cap to 160 KiB exactly once per kernel and
// device (the attribute belongs to the current device's copy of the function; a std::call_once per
// device, whichever thread gets there first, the others wait for it); device_cu_count() is the
// compute-unit count of the CURRENT device, cached per device.
constexpr int kMaxDevices = 64;
template <auto Kernel>
inline hipError_t allow_max_lds()
{
    static std::once_flag once[kMaxDevices];
    static hipError_t err[kMaxDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    std::call_once(once[dev], [dev] {
        err[dev] = hipFuncSetAttribute(reinterpret_cast<const void *>(Kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    });
    return err[dev];
}
int device_cu_count();

// The sample call's timing events handed to the MLP sampler's one launch: hipExtLaunchKernel records them as part of
// that dispatch, so no hipEventRecord call sits on the host path in front of the launch (sample_impl sets them for the
// launch and clears them after; null otherwise)
struct LaunchEvents {
    hipEvent_t start, stop;
};
extern thread_local LaunchEvents g_launch_ev;
template <typename K, typename A>
inline hipError_t launch_sampler_kernel(K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t stream, const A &args)
{
    hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, stream, g_launch_ev.start, g_launch_ev.stop, 0u, args);
    return hipGetLastError();
}

struct MlpSampleArgs {
    const float *wpack;      // packed linear layers (see mlp_sampler.hip)
    const StepPlan *plan;    // [S]
    const float *tproj;      // [S][448]
    const float *cproj;      // [B or 1][448] or null (no context / NB == 1 unconditioned)
    int64_t cproj_stride;    // 448 or 0 (shared context)
    const float *noise;      // [S+1][B][D0] or null
    float *x_out;            // [B][D0]
    float *chain;            // [S+1][B][D0] or null
    float *chain_absmax;     // [B] or null: max |x| over the chain per candidate (bits of a NaN if any)
    int64_t batch;
    int64_t global_offset;
    uint64_t seed;
    int32_t n_steps;
    int32_t mode;            // MODE_*
    int32_t clamp_x0;
    float wp1, wf;           // fp32(1 + w), fp32(w)
    float *dbg;              // debug: block 0 dumps every layer output [14][32][256] (null in production)
    // mpcd_mpc_step with the fp16 kernel: the shared context row's projection computed in the launch (cps staging)
    // instead of read from cproj (no ctx prologue launch); cproj still non-null (selects the ctx instantiation)
    int32_t ctx_fused;
    int32_t ctx_dim, n_cond, cond_dim;
    const CondLayer *cond_layers;
    CtxRowArg ctx_row;
};

int mlp_packed_floats(int d0);
void mlp_pack_weights(int d0, const float *const *lin_w, const float *const *lin_b, float *out);
hipError_t launch_mlp_sampler(int d0, int nb, const MlpSampleArgs &a, hipStream_t stream);
// fp32-accurate split-bf16 variant (mlp_x3.hip); shared or no context only
int mlp_packed_floats_x3(int d0);
void mlp_x3_force_layout(int layout);  // mpcd_mlp_force_layout
int mlp_x3_layout_of(int64_t batch, int nb);  // mpcd_mlp_layout: the layout a call of this batch runs
void mlp_pack_weights_x3(int d0, const float *const *lin_w, const float *const *lin_b, float *out);
hipError_t launch_mlp_x3(int d0, int nb, const MlpSampleArgs &a, hipStream_t stream);
// resident-weight variant (mlp_rw.hip), selected by mlp_x3's layout choice: rows = 32 or 16 per workgroup
hipError_t launch_mlp_rw(int d0, int rows, const MlpSampleArgs &a, hipStream_t stream);
// two-term fp16 variant (mlp_h2.hip, MPCD_F16X2): CFG-DDPM / eps at H*d 32 / 64, shared context; rows 32 or 16
bool mlp_h2_supports(int d0, int mode);
int mlp_packed_floats_h2(int d0);
void mlp_pack_weights_h2(int d0, const float *const *lin_w, const float *const *lin_b, float *out);
hipError_t launch_mlp_h2(int d0, int rows, const MlpSampleArgs &a, hipStream_t stream);

// Fused selection for launch_rollout_cost (single rank): see rollout.hip SelectK
constexpr int64_t kFuseClipMax = 16384;  // clip inputs up to this many floats are tested inside the selecting launch
struct RolloutSelect {
    mpcd_best *best;
    float *row_out;
    double *part_cost;
    int64_t *part_idx;
    unsigned *counter;    // zero-initialised, reset by the kernel
    int64_t n_part;       // capacity of part_* (>= ceil(batch / 64))
    int64_t offset;
    int32_t *code_out;    // optional: the clip code flags[0], written with the winner (mpcd_mpc_step's result block)
    // optional: the clip code is computed in this launch, by every workgroup, over clip_src[0, clip_n) (the
    // clip_flag_kernel test; a small batch's per-candidate chain maxima) instead of read from flag_dev
    const float *clip_src;
    int64_t clip_n;
    // optional: the result block {best, winner row, clip code} (step_out's layout) also written by the selecting
    // workgroup to mapped host memory, then *host_flag = host_seq after a system-scope fence: mpcd_mpc_step spins
    // on that word instead of a device-to-host copy and a stream synchronisation
    char *host_out;
    uint32_t *host_flag;
    uint32_t host_seq;
};
constexpr int kRolloutBlock = 64;  // candidates per rollout workgroup
