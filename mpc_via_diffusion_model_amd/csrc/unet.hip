// 1D temporal U-Net sampler — placeholder until the conv kernels land.
#include "unet.h"

namespace {
thread_local const char *g_unet_err = "";
}

int unet_prepare(const mpcd_net_desc &, size_t, const TensorLookup &, const TensorLookup &, UnetWeights &w, void *&,
                 size_t &)
{
    w.ready = false;
    g_unet_err = "UNet kernels not built yet";
    return MPCD_EUNSUP;
}

size_t unet_workspace_bytes(const mpcd_net_desc &, int64_t, int) { return 0; }

int unet_sample(const mpcd_net_desc &, const UnetWeights &, const UnetSampleArgs &, hipStream_t)
{
    g_unet_err = "UNet kernels not built yet";
    return MPCD_EUNSUP;
}

const char *unet_last_error() { return g_unet_err; }
