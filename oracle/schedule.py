"""Variance schedules and diffusion buffers (oracle; test infrastructure only).

Restates
  mpd/models/diffusion_models/helpers.py:26-37  cosine_beta_schedule (numpy fp64 -> fp32)
  mpd/models/diffusion_models/helpers.py:40-46  exponential_beta_schedule (fp32 torch)
  mpd/models/diffusion_models/diffusion_model_base.py:73-109  the 12 registered buffers
The un-vendored ``torch_robotics.to_torch`` only casts to fp32 on CPU.
"""
import numpy as np
import torch

BUFFER_NAMES = (
    "betas", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_alphas_cumprod",
    "sqrt_one_minus_alphas_cumprod", "log_one_minus_alphas_cumprod",
    "sqrt_recip_alphas_cumprod", "sqrt_recipm1_alphas_cumprod", "posterior_variance",
    "posterior_log_variance_clipped", "posterior_mean_coef1", "posterior_mean_coef2",
)


def exponential_betas(n):
    # helpers.py:40-46: beta_start * exp(a * linspace(0, n, n)), a = log(end/start)/n, fp32
    grid = torch.linspace(0, n, n)
    b0 = torch.tensor(1e-4, dtype=torch.float32)
    b1 = torch.tensor(1.0, dtype=torch.float32)
    rate = 1 / n * torch.log(b1 / b0)
    return b0 * torch.exp(rate * grid)


def cosine_betas(n, s=0.008, lo=0.0, hi=0.999):
    # helpers.py:26-37, computed in numpy fp64 then cast to fp32
    m = n + 1
    u = np.linspace(0, m, m)
    abar = np.cos(((u / m) + s) / (1 + s) * np.pi * 0.5) ** 2
    abar = abar / abar[0]
    b = 1 - (abar[1:] / abar[:-1])
    return torch.tensor(np.clip(b, a_min=lo, a_max=hi), dtype=torch.float32)


def buffers(kind, n):
    """Return dict name -> fp32 tensor[n] exactly as GaussianDiffusionModel.__init__ builds them."""
    if kind == "exponential":
        b = exponential_betas(n)
    elif kind == "cosine":
        b = cosine_betas(n)
    else:
        raise NotImplementedError(kind)
    a = 1.0 - b
    ac = torch.cumprod(a, axis=0)
    np_err = np.seterr(invalid="ignore")  # beta > 1 (exponential, some N) -> NaN, as in the reference
    acp = torch.cat([torch.ones(1), ac[:-1]])
    pv = b * (1.0 - acp) / (1.0 - ac)
    out = {
        "betas": b,
        "alphas_cumprod": ac,
        "alphas_cumprod_prev": acp,
        "sqrt_alphas_cumprod": torch.sqrt(ac),
        "sqrt_one_minus_alphas_cumprod": torch.sqrt(1.0 - ac),
        "log_one_minus_alphas_cumprod": torch.log(1.0 - ac),
        "sqrt_recip_alphas_cumprod": torch.sqrt(1.0 / ac),
        "sqrt_recipm1_alphas_cumprod": torch.sqrt(1.0 / ac - 1),
        "posterior_variance": pv,
        "posterior_log_variance_clipped": torch.log(torch.clamp(pv, min=1e-20)),
        # np.sqrt on an fp32 tensor: correctly rounded fp32 sqrt, same as torch.sqrt
        "posterior_mean_coef1": b * torch.from_numpy(np.sqrt(acp.numpy())) / (1.0 - ac),
        "posterior_mean_coef2": (1.0 - acp) * torch.from_numpy(np.sqrt(a.numpy())) / (1.0 - ac),
    }
    np.seterr(**np_err)
    return out
