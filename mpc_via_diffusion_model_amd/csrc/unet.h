// 1D temporal U-Net sampler (ConditionedTemporalUnet / TemporalUnet) — internal interface.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>

#include "../../include/mpcd.h"
#include "internal.h"

struct UnetWeights {
    bool ready = false;
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
};

using TensorLookup = std::function<const float *(const char *)>;

// dev(name): device pointer of a blob tensor; host(name): host pointer of the same tensor.
// Repacks conv weights into `pack` (device, grown as needed).
int unet_prepare(const mpcd_net_desc &d, size_t n_tensors, const TensorLookup &dev, const TensorLookup &host,
                 UnetWeights &w, void *&pack, size_t &pack_bytes);
size_t unet_workspace_bytes(const mpcd_net_desc &d, int64_t batch, int nb);
int unet_sample(const mpcd_net_desc &d, const UnetWeights &w, const UnetSampleArgs &a, hipStream_t stream);
const char *unet_last_error();
