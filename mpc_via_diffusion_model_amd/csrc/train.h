// Internal interface of the native MLP training step (train.hip); the C ABI is in mpcd_api.hip.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "common.h"

struct TrainLin {  // one nn.Linear inside the flat parameter blob: weight [n][k] at w, bias [n] at b
    int64_t w = 0, b = 0;
    int n = 0, k = 0;
};
struct TrainBlock {  // TemporalBlockMLP: la (cin -> co), lb (co -> co), lc (cond -> co)
    TrainLin la, lb, lc;
    int co = 0;
    int in0 = -1, in1 = -1;  // input: block in0's output (-1: x_noisy), concatenated with block in1's (-1: none)
};
// U-Net trunk as a tape of ops over per-row tensors [L][C] (channels-last, rows = candidates)
enum UOpKind { UOP_CONV = 0, UOP_CONVT = 1, UOP_GN = 2, UOP_MISH = 3, UOP_ADDC = 4, UOP_ADD = 5, UOP_LIN = 6 };
struct UTensor {
    int L = 1, C = 1;
};
struct UOp {
    int kind = 0;
    int in0 = -1, in1 = -1, out = -1;  // tensor ids (in1: CONV concat second input, ADDC cond [1][C], ADD addend)
    int64_t w = -1, b = -1;            // parameter offsets (weight, bias / GroupNorm affine)
    int k = 1, s = 1, p = 0, groups = 1;
};
constexpr int UT_XNOISY = 0, UT_MC = 1;  // fixed tensor ids: x_noisy [H][d], Mish(c_emb) [1][T + C]

struct TrainSpec {
    int flat = 0, temb = 0, ctx_dim = 0, base = 0, n_steps = 0;
    int64_t n_params = 0;
    float lr = 1e-3f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, ema_decay = 0.995f;
    int step_start_ema = 1000, update_ema_every = 10;
    TrainLin t1, t2, f1, f2;
    std::vector<TrainBlock> blocks;  // execution order: downs, mid, ups (MLP)
    bool unet = false;               // ConditionedTemporalUnet: the trunk is the tape below
    std::vector<UTensor> ut;
    std::vector<UOp> uops;
    int u_out = -1;                  // tensor id of the net output [H][d]
};
struct TrainBatch {
    const float *x0, *ctx, *noise, *mask;
    const int64_t *t;
    int64_t batch;
    void *stream;
};
struct Trainer;
Trainer *trainer_new(const TrainSpec &sp, const float *params_host, const float *sched_host, std::string *why);
int trainer_step(Trainer *t, const TrainBatch &b, bool update, double *loss, std::string *why);
int trainer_read(Trainer *t, int which, float *host, size_t n);
int64_t trainer_steps(Trainer *t);
void trainer_free(Trainer *t);
struct Comm;
int trainer_set_comm(Trainer *t, Comm *c);  // takes ownership; -1 if one is set already
