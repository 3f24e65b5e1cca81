/*
 * mpcd.h — C ABI of libmpcd.so, the MI355X (gfx950) diffusion-MPC hot path.
 *
 * The reference (XuehuaOvO/MPC_via_Diffusion_Model) is pure Python/PyTorch; its seam for this
 * path is a Python call, not an FFI. Each entry point below replaces one reference interface
 * (cited file:line, paths relative to the reference root); the Python package
 * mpc_via_diffusion_model_amd binds them with ctypes.
 *
 * Conventions
 *  - Every function returns 0 (MPCD_OK) or a negative mpcd_status; nothing throws across the ABI.
 *    mpcd_last_error() gives a thread-local message for the last failure on this thread.
 *  - "dev" pointers are device (HBM) pointers owned by the caller; "host" pointers are read
 *    during the call only. Weights, schedule, plan and workspace belong to the context.
 *  - Work is enqueued on the caller's HIP stream (void* hip_stream; NULL = legacy default stream)
 *    and is asynchronous unless stated otherwise. One context per device; not thread-safe.
 *  - A context owns workspace (plan, projections, U-Net activations, reduction counters) that
 *    consecutive calls reuse: issue a context's calls on ONE stream, or order the streams yourself
 *    (hipStreamWaitEvent) before switching. The cached step plan / time projections are the exception:
 *    a call on another stream waits for them by itself.
 *  - All trajectory tensors are fp32 row-major [B][H][d] (candidate, horizon, action dim), the
 *    layout of the reference's x in cart_pole_sample_loop (diffusion_model_base.py:188-189).
 */
#ifndef MPCD_H
#define MPCD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mpcd_ctx mpcd_ctx;

enum mpcd_status {
    MPCD_OK = 0,
    MPCD_EINVAL = -1,   /* bad argument / shape */
    MPCD_EHIP = -2,     /* HIP runtime error */
    MPCD_ESTATE = -3,   /* missing net / schedule, or call out of order */
    MPCD_ENOMEM = -4,
    MPCD_EUNSUP = -5,   /* configuration the kernels do not implement */
    MPCD_ENONFINITE = -6, /* mpcd_mpc_step: no candidate has a finite cost (NaN / Inf samples or rollout) -
                             the result block is still written; see mpcd_last_step_flags */
};

enum mpcd_net_kind {
    MPCD_NET_MLP = 1,   /* build-defined CFG MLP noise-net: PointUnet stack on [B, H*d] (temporal_unet.py:451-550) */
    MPCD_NET_UNET = 2,  /* ConditionedTemporalUnet (temporal_unet.py:189-358) or TemporalUnet (:28-187) */
};

/* GEMM numerics of the noise-net.
 * MPCD_F32:   exact fp32 MFMA (v_mfma_f32_16x16x4_f32: one rounding per product, an fmaf chain).
 * MPCD_F16:   fp16 GEMM operands with fp32 accumulation on v_mfma_f32_16x16x32_f16 (SURVEY cfg 5,
 *             "fp16 hidden with MFMA GEMM"); U-Net only (an MLP net returns MPCD_EUNSUP).
 * MPCD_F32X3: fp32-accurate split-bf16 MFMA (MLP and U-Net): each fp32 operand = three bf16 terms, the six
 *             partial products >= 2^-16 of the leading one accumulated in fp32 (error at the level of
 *             the fp32 MFMA's). MLP: needs a context shared by all candidates (or none); a
 *             per-candidate context runs the MPCD_F32 kernel.
 * MPCD_F16X2: two-term fp16 MFMA (MLP: csrc/mlp_h2.hip; U-Net: the fused P = 2 program) - NOT fp32 arithmetic:
 *             each operand = hi + lo (two fp16, the weights scaled per layer by an exact power of two, the
 *             activations unscaled), three products per 32-k chunk accumulated in fp32. 22 significant bits per
 *             operand (fp32: 24) and the fp16 range: an activation above 65504 becomes a NaN sample (mpcd_mpc_step
 *             then re-runs the step in MPCD_F32X3, see mpcd_force_f32x3), activations below 2^-14 keep an
 *             absolute, not relative, precision of 2^-25. Used for the CFG-DDPM sampler and the eps forward (MLP at
 *             H*d = 32 / 64 with a shared context); every other case (unclamped DDIM, whose unbounded x leaves
 *             the fp16 range; per-candidate contexts; H*d = 128) runs the MPCD_F32X3 kernels of the same net. */
enum mpcd_dtype { MPCD_F32 = 0, MPCD_F16 = 1, MPCD_F32X3 = 2, MPCD_F16X2 = 3 };

typedef struct {
    int32_t kind;          /* mpcd_net_kind */
    int32_t state_dim;     /* d: channels of the denoised trajectory (actions per horizon point) */
    int32_t horizon;       /* H (MLP: input width H*d; UNet: H % 4 == 0) */
    int32_t context_dim;   /* C: conditioning width (0 = TemporalUnet with conditioning None) */
    int32_t base_dim;      /* unet_input_dim / dim, 32 */
    int32_t n_mults;       /* len(dim_mults), 3 for UNET_DIM_MULTS[0] = (1, 2, 4) */
    int32_t mults[4];
    int32_t time_emb_dim;  /* 32 */
    int32_t cfg_masked;    /* 1: 4-arg net with the CFG context mask (ConditionedTemporalUnet :296-300);
                              0: 3-arg TemporalUnet (context concatenated unmasked when C > 0) */
    int32_t dtype;         /* mpcd_dtype of the hidden activations/GEMM operands */
} mpcd_net_desc;

/* Parameter blob = every parameter of the torch module, flattened row-major, concatenated in the
 * order mpcd_net_param_info() enumerates (= the module's state_dict() order, which is the
 * reference's for the U-Nets, e.g. "time_mlp.encoder.1.weight", "downs.0.0.blocks.0.block.0.weight").
 * Replaces GaussianDiffusionModel(model=...) + load_state_dict (Diffusion_MPC_Inference.py:211-222). */
int mpcd_net_param_count(const mpcd_net_desc *desc, int32_t *n_tensors, int64_t *n_floats);
int mpcd_net_param_info(const mpcd_net_desc *desc, int32_t i, char *name, size_t name_cap,
                        int32_t *ndim, int64_t shape[4]);

int mpcd_create(int device, mpcd_ctx **out);
void mpcd_destroy(mpcd_ctx *ctx);
const char *mpcd_last_error(void);

/* Upload and repack weights into the kernels' layouts (blocking). */
int mpcd_load_net(mpcd_ctx *ctx, const mpcd_net_desc *desc, const float *blob_host, size_t n_floats);

/* The 12 diffusion buffers, fp32, each [n_steps], in GaussianDiffusionModel's registration order
 * (diffusion_model_base.py:87-109): betas, alphas_cumprod, alphas_cumprod_prev, sqrt_alphas_cumprod,
 * sqrt_one_minus_alphas_cumprod, log_one_minus_alphas_cumprod, sqrt_recip_alphas_cumprod,
 * sqrt_recipm1_alphas_cumprod, posterior_variance, posterior_log_variance_clipped,
 * posterior_mean_coef1, posterior_mean_coef2.
 * posterior_std_host: optional [n_steps] = sqrt(exp(posterior_log_variance_clipped)) as the caller's
 * fp32 math computes it (sample_functions.py:35-37); NULL = computed here with expf/sqrtf. */
int mpcd_set_schedule(mpcd_ctx *ctx, const float *tables_host, int32_t n_steps, const float *posterior_std_host);

enum mpcd_sampler {
    MPCD_DDPM_CFG = 0,  /* run_CFG + ddpm_cart_pole_sample_fn (diffusion_model_base.py:394-418, sample_functions.py:17-44) */
    MPCD_DDIM_CFG = 1,  /* build-defined CFG-DDIM */
    MPCD_DDIM = 2,      /* ddim_sample with a 3-arg net (diffusion_model_base.py:239-314), eta = 0 */
};

typedef struct {
    const float *context;      /* dev [B][C] normalised context, or [1][C] if context_shared; NULL if C == 0 */
    int32_t context_shared;    /* 1: one context row for every candidate (one x0 per control step) */
    int32_t sampler;           /* mpcd_sampler */
    int64_t batch;             /* B candidates handled by this call (this rank's shard) */
    double w;                  /* CFG weight (context_weight of run_CFG) */
    int32_t n_wo_noise;        /* n_diffusion_steps_without_noise (DDPM) */
    int32_t ddim_steps;        /* DDIM sampling_timesteps; 0 = reference n_steps // 5 (:252) */
    int32_t clamp_x0;          /* DDIM only; DDPM always clamps (clip_denoised, :172-173) */
    int32_t n_ddim_times;      /* length of ddim_times, 0 = derive the grid here */
    const int32_t *ddim_times; /* host, optional: the reference's time list [T-1, ..., 0, -1] (:255-258) */
    uint64_t seed;             /* Philox4x32-10 key (throughput mode) */
    int64_t global_offset;     /* global index of candidate 0 (Philox counter; sharding-invariant) */
    const float *noise;        /* dev [S+1][B][H][d] injected noise (parity mode) or NULL -> Philox;
                                  slice 0 = x_T, slice k = the draw of denoise step k */
    float *x_out;              /* dev [B][H][d] final normalised sample */
    float *chain_out;          /* dev [S+1][B][H][d] or NULL (run_CFG return_chain, :403-415) */
    float *chain_absmax;       /* dev [B] or NULL: per candidate, max |x| over every chain slice x_T .. x_0
                                  (NaN if any element is NaN) - what LimitsNormalizer's global clip test
                                  sees when the caller unnormalises the whole chain (see mpcd_clip_rule) */
} mpcd_sample_args;

/* The sampler's in-kernel noise stream (Philox4x32-10 keyed by seed, global candidate index, slice,
 * element quad) for candidates [global_offset, global_offset + n_cand): out dev [n_slices][n_cand][flat]
 * fp32, slice 0 = x_T, slice k = the draw of denoise step k (what `noise` would have to hold to replay
 * a Philox run in injected-noise mode). flat = H*d, a multiple of 4. */
int mpcd_philox_noise(uint64_t seed, int64_t global_offset, int64_t n_cand, int32_t n_slices, int32_t flat,
                      float *out, void *hip_stream);

/* Number of denoise steps S a call makes (DDPM: N + n_wo_noise; DDIM: grid pairs). */
int mpcd_sample_steps(mpcd_ctx *ctx, const mpcd_sample_args *args, int32_t *n_steps);
int mpcd_sample(mpcd_ctx *ctx, const mpcd_sample_args *args, void *hip_stream);

/* One noise-net forward at diffusion time t (the model(x, t, context, mask) calls of
 * p_mean_variance_CFG, diffusion_model_base.py:166-168): x dev [B][H][d]; eps_cond dev [B][H][d] =
 * net(x, t, ctx, mask = 0); eps_uncond dev [B][H][d] = net(x, t, ctx, mask = 1) for a cfg_masked net
 * (NULL for a 3-arg net, whose single output goes to eps_cond). */
int mpcd_eps(mpcd_ctx *ctx, const float *x, int32_t t, const float *context, int32_t context_shared, int64_t batch,
             float *eps_cond, float *eps_uncond, void *hip_stream);

/* --- rollout / cost / selection --- */
enum mpcd_system {
    MPCD_SYS_CARTPOLE_LIN5 = 0,  /* EulerForwardCartpole_virtual, Cart_Diffusion_inference.py:168-197 */
    MPCD_SYS_CARTPOLE_NL5 = 1,   /* nonlinear Euler, nmpc_multi_process_collect_data.py:121-137 */
    MPCD_SYS_CARTPOLE_ZOH4 = 2,  /* linear ZOH, Diffusion_MPC_Inference.py:39-84 */
    MPCD_SYS_DOUBLE_INT2D = 3,   /* build-defined */
    MPCD_SYS_PENDULUM = 4,       /* build-defined */
    MPCD_SYS_QUADROTOR12 = 5,    /* build-defined */
};
enum mpcd_cost_kind {
    MPCD_COST_CANONICAL = 0,     /* J = q(x0) + sum_k [q(x_{k+1}) + r(u_k)], terminal P (nmpc...py:158-172) */
    MPCD_COST_CALMPC = 1,        /* calMPCCost quirks (Cart_Diffusion_inference.py:247-283) */
};

typedef struct {
    int32_t system;      /* mpcd_system */
    int32_t cost_kind;   /* mpcd_cost_kind */
    int32_t n_x, n_u;    /* n_u must equal the net's state_dim */
    double params[24];   /* dynamics constants, layout per system (mpc_via_diffusion_model_amd/systems.py) */
    double Q[12], R[4], P[12], x_ref[12];   /* diagonal weights and set-point, fp64 */
} mpcd_system_desc;

/* Global clip flag of LimitsNormalizer.unnormalize (normalization.py:160-162): *flag_dev = 1 iff
 * x.max() > 1+1e-4 or x.min() < -1-1e-4 over the n values, with torch's NaN semantics (a NaN anywhere
 * makes max/min NaN and both tests false: flag 0). Also valid over mpcd_sample's chain_absmax values.
 * Sharded callers max-reduce the per-rank flags (a NaN on any rank is reported as flag value 2, which
 * a max-reduction keeps: only 1 means clip). */
int mpcd_clip_flag(mpcd_ctx *ctx, const float *x, int64_t n, int32_t *flag_dev, void *hip_stream);

/* Unnormalise (LimitsNormalizer.unnormalize, normalization.py:156-167; clip iff the GLOBAL max/min of
 * u_norm leaves [-1-1e-4, 1+1e-4]) then roll out and cost every candidate in fp64, one thread each.
 * x0_host [n_x] fp64; u_norm dev [B][H][n_u]; umin/umax host [n_u] fp32 (dataset limits);
 * clip_flag_dev: dev int32 from mpcd_clip_flag (e.g. OR-reduced over ranks), or NULL = computed here
 * from u_norm; cost_out dev [B] fp64. Replaces calMPCCost / the MPC objective evaluated per sample. */
int mpcd_rollout_cost(mpcd_ctx *ctx, const mpcd_system_desc *sys, const double *x0_host, const float *u_norm,
                      const float *umin_host, const float *umax_host, int64_t batch, int32_t horizon,
                      const int32_t *clip_flag_dev, double *cost_out, void *hip_stream);

/* Unnormalise only: out = ((x+1)/2)*(max-min)+min in fp32 over [n_rows][dim], with the global clip
 * rule (clip_flag_dev as above; NULL = computed from x). dim <= 16. */
int mpcd_unnormalize(mpcd_ctx *ctx, const float *x, int64_t n_rows, int32_t dim, const float *min_host,
                     const float *max_host, const int32_t *clip_flag_dev, float *out, void *hip_stream);

typedef struct {
    double cost;         /* +inf if every cost is NaN */
    int64_t index;       /* index_offset + position; lowest index on ties; NaN costs rank as +inf */
} mpcd_best;

/* Device argmin over cost[n] (torch.argmin(cost_all), inference_(mpd).py:335-338). best_dev is a
 * device pointer to one mpcd_best. */
int mpcd_argmin(mpcd_ctx *ctx, const double *cost, int64_t n, int64_t index_offset, mpcd_best *best_dev,
                void *hip_stream);

/* ---- Closed loop on the device: M plant states advanced together, each with its
 * own group of `group` consecutive candidates, no host round trip inside the loop
 * (Cart_Diffusion_inference.py:405-512 runs one state at a time on the host). */

/* Per-group clip flags: flags_dev[g] = mpcd_clip_flag's code over x[g*group_elems, (g+1)*group_elems)
 * (LimitsNormalizer's rule applied to each state's own candidate batch, or to its candidates'
 * chain_absmax values: 1 = clip). */
int mpcd_clip_flags(mpcd_ctx *ctx, const float *x, int64_t n_groups, int64_t group_elems, int32_t *flags_dev,
                    void *hip_stream);

/* normalize_condition of n_states device fp64 states [n_states][dim] (normalization.py:149-154 in fp64,
 * then the net's .float()): ctx_out dev fp32 [n_states][dim]. min/max host fp32 [dim], dim <= 16. */
int mpcd_normalize_states(mpcd_ctx *ctx, const double *x_dev, int64_t n_states, int32_t dim, const float *min_host,
                          const float *max_host, float *ctx_out, void *hip_stream);

/* mpcd_rollout_cost with one start state per group: candidate b starts from x0_dev[b / group] (dev fp64
 * [batch/group][n_x]) and uses flags_dev[b / group]. batch % group == 0. */
int mpcd_rollout_cost_grouped(mpcd_ctx *ctx, const mpcd_system_desc *sys, const double *x0_dev, int64_t group,
                              const float *u_norm, const float *umin_host, const float *umax_host, int64_t batch,
                              int32_t horizon, const int32_t *flags_dev, double *cost_out, void *hip_stream);

/* One control step for n_states plant states (A15 + the plant step): for state m pick the candidate of
 * [m*group, (m+1)*group) with the lowest cost (NaN = +inf, lowest index on ties) or, select_first != 0,
 * the group's first one (the reference scripts' n_samples = 1 use); unnormalise its u[0] with
 * flags_dev[m]; round it to `decimals` places (the reference's round(u, 4); < 0 = no rounding); then
 * x_dev[m] <- f(x_dev[m], u0) in fp64 with the system's dynamics (in place). Outputs (device):
 * u_applied [n_states][n_u] fp64, best_index [n_states] int64 (global candidate index), best_cost fp64. */
int mpcd_control_step(mpcd_ctx *ctx, const mpcd_system_desc *sys, double *x_dev, int64_t n_states, int64_t group,
                      const float *u_norm, int32_t horizon, const double *cost, const float *umin_host,
                      const float *umax_host, const int32_t *flags_dev, int32_t select_first, int32_t decimals,
                      double *u_applied, int64_t *best_index, double *best_cost, void *hip_stream);

/* ---- Candidate-batch data parallelism over RCCL / xGMI. One process per GPU, one
 * communicator per context; rank r owns global candidates [r*B_local, (r+1)*B_local). The reference has
 * no distributed code: these entry points are new design, not replacements. */
#define MPCD_COMM_ID_BYTES 128
/* Rank 0 creates the id (ncclGetUniqueId) and ships its 128 bytes to every rank out of band. */
int mpcd_comm_unique_id(void *id_out);
int mpcd_comm_init(mpcd_ctx *ctx, int32_t nranks, int32_t rank, const void *id);
/* Loopback communicator: `nranks` VIRTUAL ranks = nranks contexts on the same device in one process,
 * each context driven by its own host thread, joined by a caller-chosen group_key. The collectives are
 * device copies ordered by HIP events plus a host rendezvous of the member threads (120 s timeout), so
 * mpcd_select / mpcd_mpc_step run their N-rank code (rank offsets, gathered-cost order, owner-row sum,
 * flag max-reduction) on one GPU: the single-GPU rehearsal and test of the RCCL path. */
int mpcd_comm_init_loopback(mpcd_ctx *ctx, int32_t nranks, int32_t rank, uint64_t group_key);

/* ---- native training step: GaussianDiffusionModel.loss / p_losses with CFG context
 * dropout (diffusion_model_base.py:434-467), WeightedL2 (helpers.py:71-99), backward, torch.optim.Adam
 * (trainer.py:152) and the EMA model (trainer.py:70-88, 302-308), on the device in fp32. The CFG MLP net and
 * ConditionedTemporalUnet (MPCD_NET_UNET with cfg_masked; training always runs in fp32 whatever desc->dtype). The random draws of p_losses (t ~ randint, noise ~ randn_like, context_mask ~
 * bernoulli(drop_prob)) are inputs, so a caller reproduces the reference's RNG stream exactly. */
typedef struct mpcd_trainer mpcd_trainer;
typedef struct {
    float lr, beta1, beta2, eps; /* Adam (torch defaults: 0.9, 0.999, 1e-8) */
    float ema_decay;             /* EMA beta (trainer default 0.995) */
    int32_t step_start_ema;      /* before this step the EMA model is reset to the model (trainer: 1000) */
    int32_t update_ema_every;    /* EMA update period in steps (trainer: 10) */
} mpcd_train_cfg;
/* params: the net's parameters in mpcd_net_param_info() order; the schedule's sqrt(abar) and
 * sqrt(1 - abar) [n_steps] (q_sample). The EMA model starts as a copy of params. */
int mpcd_trainer_create(const mpcd_net_desc *desc, const float *params, size_t n_floats, const mpcd_train_cfg *cfg,
                        const float *sqrt_alphas_cumprod, const float *sqrt_one_minus_alphas_cumprod, int32_t n_steps,
                        mpcd_trainer **out);
/* One batch (device pointers): x0 [B][H*d] normalised trajectories, context [B][C], t [B] (int64, < n_steps),
 * noise [B][H*d], context_mask [B] (1 = context dropped); t outside [0, n_steps) is clamped on the device (the
 * Python wrapper rejects it). update = 0: the loss only (p_losses forward);
 * 1: loss, backward, Adam step, EMA update. Blocks until done; *loss = mean((eps_pred - noise)^2). */
int mpcd_trainer_step(mpcd_trainer *tr, const float *x0, const float *context, const int64_t *t, const float *noise,
                      const float *context_mask, int64_t batch, int32_t update, double *loss, void *hip_stream);
/* which: 0 parameters, 1 EMA parameters, 2 last gradients, 3 Adam exp_avg, 4 Adam exp_avg_sq (host copy) */
int mpcd_trainer_params(mpcd_trainer *tr, int32_t which, float *host_out, size_t n_floats);
/* Data-parallel training: each rank steps on its own rows; the flat gradient is sum-all-reduced over the
 * communicator and divided by nranks before Adam (DistributedDataParallel's averaging), so all ranks keep
 * identical parameters and EMA. RCCL (one process per GPU; id from mpcd_comm_unique_id) or an in-process
 * loopback group of nranks trainers on one GPU, each stepped from its own host thread. */
int mpcd_trainer_comm_init(mpcd_trainer *tr, int32_t nranks, int32_t rank, const void *unique_id);
int mpcd_trainer_comm_init_loopback(mpcd_trainer *tr, int32_t nranks, int32_t rank, uint64_t group_key);
void mpcd_trainer_destroy(mpcd_trainer *tr);
int mpcd_comm_info(mpcd_ctx *ctx, int32_t *nranks, int32_t *rank);  /* 1, 0 without mpcd_comm_init */
/* recv [nranks * count_per_rank] (rank order); without a communicator: a device copy. */
int mpcd_allgather_f32(mpcd_ctx *ctx, const float *send, float *recv, size_t count_per_rank, void *hip_stream);
int mpcd_allgather_f64(mpcd_ctx *ctx, const double *send, double *recv, size_t count_per_rank, void *hip_stream);
int mpcd_broadcast_f32(mpcd_ctx *ctx, float *buf, size_t count, int32_t root, void *hip_stream);
int mpcd_allreduce_max_i32(mpcd_ctx *ctx, int32_t *buf, size_t count, void *hip_stream);  /* OR of clip flags */
/* The per-control-step exchange, device-resident end to end (no host round trip): all-gather the fp64
 * costs into costs_all [nranks * n_local], global argmin (torch.argmin(cost_all), inference_(mpd).py:335-338;
 * NaN = +inf, lowest global index on ties) into *best_dev, and the winner's row [row_len] (its normalised
 * [H][d] trajectory) into row_out on every rank (owner writes it, the others zeros, sum all-reduce). */
int mpcd_select(mpcd_ctx *ctx, const double *cost_local, int64_t n_local, const float *rows_local, int32_t row_len,
                double *costs_all, mpcd_best *best_dev, float *row_out, void *hip_stream);

/* ---- One control step in one call: the whole per-step path of Diffusion_MPC_Inference.py:229-262 /
 * Cart_Diffusion_inference.py:439-470 (normalize_condition -> run_CFG -> unnormalize_states -> cost of
 * every candidate -> argmin -> applied action) for this rank's shard, plus the exchange of mpcd_select
 * when the context has a communicator. Everything stays on the device until the result block leaves it: on one
 * rank the selecting rollout workgroup writes it to mapped pinned host memory followed by a completion word the
 * call spins on (no copy launch, no stream-synchronisation wake-up; every kernel's device writes precede that
 * word); with a communicator one D2H copy and a stream synchronisation. best_host / u_best_host are valid on
 * return either way. */
/* The reference scripts call run_CFG(..., return_chain=True) and unnormalise the WHOLE chain
 * (Cart_Diffusion_inference.py:450-463, Diffusion_MPC_Inference.py:232-247), so the clip test sees x_T
 * ~ N(0, 1) as well and practically always clips. MPCD_CLIP_CHAIN reproduces that (the default);
 * MPCD_CLIP_FINAL tests the final samples only (a caller that unnormalises just x_0); MPCD_CLIP_NONE: the
 * caller has proven the final-only flag 0 (DDPM whose last posterior mean cannot leave [-1, 1]). */
enum mpcd_clip_rule { MPCD_CLIP_CHAIN = 0, MPCD_CLIP_FINAL = 1, MPCD_CLIP_NONE = 2 };

typedef struct {
    const mpcd_system_desc *sys;   /* n_u == the net's state_dim */
    const double *x0;              /* host [n_x] fp64 plant state */
    const float *ctx_min, *ctx_max; /* host [C] condition limits: ctx = fp32(2*((x0-min)/fp32(max-min)) - 1) in fp64
                                      (LimitsNormalizer.normalize, normalization.py:149-154) */
    const float *act_min, *act_max; /* host [d] action limits (LimitsNormalizer.unnormalize, :156-167) */
    mpcd_sample_args sample;       /* .context / .context_shared are ignored (the normalised x0 is the shared
                                      context); .batch = B_local; .global_offset = rank * B_local; .x_out required;
                                      .chain_absmax is set by the call itself under MPCD_CLIP_CHAIN */
    int32_t clip_rule;             /* mpcd_clip_rule: which tensor LimitsNormalizer's global clip test runs over */
    double *cost_local;            /* dev [batch] fp64 costs of this rank's candidates (out) */
    double *costs_all;             /* dev [nranks * batch] all costs (out), needed with a communicator, else unused */
} mpcd_step_args;

/* Ordering: best_host / u_best_host are complete when the call returns (one rank: the call spins on a completion word
 * the selecting workgroup writes to mapped host memory after the result block; with a communicator: a stream
 * synchronisation). The DEVICE outputs (sample.x_out, cost_local, costs_all) are ordered only on hip_stream: read them
 * from another stream or from the host after a stream synchronisation or an event.
 * best_host: global winner (index over all ranks); u_best_host: host [H*d] fp32, the winner's
 * UNnormalised trajectory (u_best[0] is the applied action before the reference's rounding).
 * Returns MPCD_ENONFINITE (outputs written) when the winning cost is not finite, i.e. every candidate of
 * every rank is NaN / Inf - garbage is never returned as a normal result. */
int mpcd_mpc_step(mpcd_ctx *ctx, const mpcd_step_args *args, mpcd_best *best_host, float *u_best_host,
                  void *hip_stream);

/* Failure-detection flags of the last mpcd_mpc_step on this context (read after it returned):
 * bit 0 (MPCD_STEP_CLIPPED): LimitsNormalizer's global clip was applied; bit 1 (MPCD_STEP_NAN_SAMPLES): some
 * candidate's tested tensor (its chain under MPCD_CLIP_CHAIN, its final sample under MPCD_CLIP_FINAL) holds a
 * NaN on some rank - the reference's torch max()/min() are then NaN and nothing is clipped; bit 2
 * (MPCD_STEP_NONFINITE_WINNER): no finite cost (the call returned MPCD_ENONFINITE); bit 3 (MPCD_STEP_F32X3_RERUN): an
 * MPCD_F16X2 net's step left the fp16 range (NaN samples or no finite cost, one rank) and was re-run with the net's
 * split-bf16 programs - the other bits and the outputs are the re-run's. */
enum { MPCD_STEP_CLIPPED = 1, MPCD_STEP_NAN_SAMPLES = 2, MPCD_STEP_NONFINITE_WINNER = 4, MPCD_STEP_F32X3_RERUN = 8 };
int mpcd_last_step_flags(mpcd_ctx *ctx, int32_t *flags);

/* U-Net conv tilings (MPCD_F32X3 / MPCD_F16). Each conv launch picks rows-per-workgroup x register tile
 * x persistent-or-not among candidates by timing them once per layer shape and batch, and each
 * ResidualTemporalBlock picks fused-or-not the same way. This process-wide override makes the choice
 * deterministic, so a caller can run EVERY candidate on its own batch (they are bit-identical: the
 * K order and the GroupNorm summation order do not depend on the tiling):
 *   conv_pick  -1 = measured (default); i >= 0 = candidate (i mod count) for every conv, blocks unfused
 *              unless block_pick says otherwise;
 *   block_pick -1 = measured; -2 = never fuse; i >= 0 = fused candidate (i mod count) for every block. */
int mpcd_unet_force_tiling(int32_t conv_pick, int32_t block_pick);
/* MLP split-bf16 sampler workgroup layout (rows x waves), process-wide: -1 = by batch size (default: rw32, or
 * rw16 when 32-row workgroups would leave CUs idle); 0 = 32x8; 1 = 16x8; 2 = 16x4 (two 4-wave workgroups per
 * CU where their LDS fits, else 16x8); 3 / 4 = rw32 / rw16 (csrc/mlp_rw.hip: 32 / 16 rows on 4 waves, the
 * 128-wide layers' weights resident in registers for the whole launch). All layouts compute the same sums in
 * the same order (bit-identical results). */
int mpcd_mlp_force_layout(int32_t layout);
/* The layout (0..4 as above) an MPCD_F32X3 MLP sample call of `batch` candidates runs on the current device
 * (cfg_masked: CFG net, two rows per candidate). */
int mpcd_mlp_layout(int64_t batch, int32_t cfg_masked, int32_t *layout_out);
/* Which kernel an mpcd_sample / mpcd_mpc_step call with this sampler and `batch` candidates (shared context) runs
 * on this context's MLP, on its device: out[0] = 0 exact fp32 (mlp_sample_kernel), 1 split bf16 (mlp_x3_kernel /
 * mlp_rw_kernel), 2 two-term fp16 (mlp_h2_kernel); out[1] = the bf16x3 layout (as mpcd_mlp_layout) or -1;
 * out[2] = rows per workgroup (32 or 16). MPCD_EUNSUP on a U-Net context. */
int mpcd_mlp_form(mpcd_ctx *ctx, int32_t sampler, int64_t batch, int32_t out[3]);
/* on != 0: an MPCD_F16X2 net runs its split-bf16 (MPCD_F32X3) programs for every call on this context until turned
 * off again (mpcd_mpc_step does this by itself for one re-run when an MPCD_F16X2 step's samples come back with a NaN
 * or without a finite cost: the fp16 range was left; MPCD_STEP_F32X3_RERUN flags it). */
int mpcd_force_f32x3(mpcd_ctx *ctx, int32_t on);
/* U-Net execution form, process-wide. The whole-network form (csrc/unet_fused.hip: every conv of one denoise
 * step in ONE launch, a workgroup per few candidates, activations in LDS) covers the CFG samplers and the
 * two-branch eps of ConditionedTemporalUnet(base 32, dim_mults (1, 2, 4)) at H = 32 / 64 with the MPCD_F32X3
 * or MPCD_F16 numerics; everything else runs layer by layer (one launch per conv). 0 = automatic (the fused
 * form where it applies; env MPCD_UNET_FUSED=0 turns it off), 1 = layer by layer, 2 = fused (a sample / eps
 * call it does not cover returns MPCD_EUNSUP). */
int mpcd_unet_force_path(int32_t path);
/* Which form an mpcd_sample call with this sampler (mpcd_sampler) takes on this context's U-Net under the
 * current mpcd_unet_force_path / MPCD_UNET_FUSED settings: out[0] = 1 whole-network fused launch per denoise
 * step / 0 layer by layer, out[1] = GEMM operand planes (0 exact fp32, 1 fp16, 3 split bf16), out[2] = rows
 * (candidate x CFG branch) and out[3] = waves per workgroup of the fused launch. MPCD_EUNSUP on an MLP
 * context. */
int mpcd_unet_form(mpcd_ctx *ctx, int32_t sampler, int32_t out[4]);
#define MPCD_UNET_MAX_CONV_TILINGS 12   /* 6 rows-per-workgroup values x {tiled, persistent} */
#define MPCD_UNET_MAX_BLOCK_TILINGS 6

/* Timing of the last mpcd_sample's main kernel (HIP events on the call's stream), milliseconds.
 * Blocks until that kernel has finished. */
int mpcd_last_sample_ms(mpcd_ctx *ctx, float *ms);
/* Mean of that timing over the last n sample calls (1 <= n <= 256 and <= the calls made): a timed control loop reads
 * it once afterwards instead of one mpcd_last_sample_ms per step. Blocks until the last of them has finished. */
int mpcd_sample_ms_mean(mpcd_ctx *ctx, int32_t n, float *ms);

#ifdef __cplusplus
}
#endif
#endif /* MPCD_H */
