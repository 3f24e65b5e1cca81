// 1D temporal U-Net sampler (ConditionedTemporalUnet / TemporalUnet) — internal interface.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <vector>

#include "../../include/mpcd.h"
#include "internal.h"

// One fused conv launch of the U-Net (see unet.hip for the op list).
struct ConvLayer {
    int kind;          // CONV_SAME5 / CONV_DOWN3 / CONV_UP4 / CONV_PW1
    int cin, cout;     // total input channels (a + b concat), output channels
    int coutp;         // cout padded to a multiple of 16 (MFMA n-tiles)
    int cinp;          // cin padded to a multiple of 4 (first layer: d -> 4/8)
    int kpad;          // packed K per parity, multiple of 16
    const float *w;    // packed A operand (device), [parities][cout/16][kpad/16][64][4]
    const float *bias; // [cout]
    const float *gn_w, *gn_b;  // GroupNorm affine or null
    int groups;
    int cond_off;      // column of this block in tproj/cproj, -1 = none
};

struct UnetWeights {
    bool ready = false;
    int n_layers = 0;
    std::vector<ConvLayer> layers;  // in execution order (see unet.hip build_plan)
};

struct UnetSampleArgs {
    const StepPlan *plan;
    const StepPlan *plan_host;
    const float *tproj;
    const float *cproj;
    int64_t cproj_stride;
    int32_t cond_total;
    const float *noise;
    float *x_out;
    float *chain;
    int64_t batch;
    int64_t global_offset;
    uint64_t seed;
    int32_t n_steps;
    int32_t mode;
    int32_t clamp_x0;
    float wp1, wf;
    void *workspace;
    float *eps_cond, *eps_uncond;  // MODE_EPS / MODE_EPS1 outputs
    const float *x_in;             // MODE_EPS / MODE_EPS1 input
};

using TensorLookup = std::function<const float *(const char *)>;

// dev(name): device pointer of a blob tensor; host(name): host pointer of the same tensor.
// Repacks conv weights into `pack` (device, grown as needed).
int unet_prepare(const mpcd_net_desc &d, size_t n_tensors, const TensorLookup &dev, const TensorLookup &host,
                 UnetWeights &w, void *&pack, size_t &pack_bytes);
size_t unet_workspace_bytes(const mpcd_net_desc &d, int64_t batch, int nb);
int unet_sample(const mpcd_net_desc &d, const UnetWeights &w, const UnetSampleArgs &a, hipStream_t stream);
const char *unet_last_error();
