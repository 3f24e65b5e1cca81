"""Diffusion schedule tables, computed on the host exactly as the reference does (fp32 torch CPU ops).

mpd/models/diffusion_models/helpers.py:26-46 (cosine / exponential betas) and
diffusion_model_base.py:80-109 (the 12 registered buffers). When a trained state dict is loaded
its own buffers are used instead (load_state_dict overwrites them in the reference too).
"""
import numpy as np
import torch

TABLE_ORDER = ("betas", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_alphas_cumprod",
               "sqrt_one_minus_alphas_cumprod", "log_one_minus_alphas_cumprod", "sqrt_recip_alphas_cumprod",
               "sqrt_recipm1_alphas_cumprod", "posterior_variance", "posterior_log_variance_clipped",
               "posterior_mean_coef1", "posterior_mean_coef2")


def betas(kind, n_steps):
    if kind == "exponential":
        x = torch.linspace(0, n_steps, n_steps)
        lo, hi = torch.tensor(1e-4, dtype=torch.float32), torch.tensor(1.0, dtype=torch.float32)
        return lo * torch.exp(1 / n_steps * torch.log(hi / lo) * x)
    if kind == "cosine":
        s, m = 0.008, n_steps + 1
        g = np.linspace(0, m, m)
        ac = np.cos(((g / m) + s) / (1 + s) * np.pi * 0.5) ** 2
        ac = ac / ac[0]
        return torch.tensor(np.clip(1 - (ac[1:] / ac[:-1]), a_min=0, a_max=0.999), dtype=torch.float32)
    raise ValueError(f"unknown variance schedule {kind!r}")


def tables(kind, n_steps):
    b = betas(kind, n_steps)
    alpha = 1.0 - b
    ac = torch.cumprod(alpha, axis=0)
    acp = torch.cat([torch.ones(1), ac[:-1]])
    pv = b * (1.0 - acp) / (1.0 - ac)
    with np.errstate(invalid="ignore"):  # beta > 1 (exponential, some N) -> NaN, as in the reference
        sq_acp, sq_alpha = np.sqrt(acp.numpy()), np.sqrt(alpha.numpy())
    return {
        "betas": b, "alphas_cumprod": ac, "alphas_cumprod_prev": acp, "sqrt_alphas_cumprod": torch.sqrt(ac),
        "sqrt_one_minus_alphas_cumprod": torch.sqrt(1.0 - ac), "log_one_minus_alphas_cumprod": torch.log(1.0 - ac),
        "sqrt_recip_alphas_cumprod": torch.sqrt(1.0 / ac), "sqrt_recipm1_alphas_cumprod": torch.sqrt(1.0 / ac - 1),
        "posterior_variance": pv, "posterior_log_variance_clipped": torch.log(torch.clamp(pv, min=1e-20)),
        "posterior_mean_coef1": b * torch.from_numpy(sq_acp) / (1.0 - ac),
        "posterior_mean_coef2": (1.0 - acp) * torch.from_numpy(sq_alpha) / (1.0 - ac),
    }


def posterior_std(tabs):
    """sqrt(exp(posterior_log_variance_clipped)) with torch fp32 ops (sample_functions.py:35-44)."""
    return torch.sqrt(torch.exp(tabs["posterior_log_variance_clipped"]))


def pack(tabs):
    """12 x N contiguous fp32 in the ABI order."""
    return torch.stack([tabs[k].to(torch.float32) for k in TABLE_ORDER]).contiguous()


def is_finite(tabs):
    return all(bool(torch.isfinite(tabs[k]).all()) for k in TABLE_ORDER)


def ddim_times(n_steps, sampling_steps=None):
    """The reference's DDIM time list [T-1, ..., 0, -1] (diffusion_model_base.py:251-258), via torch."""
    s = n_steps // 5 if sampling_steps is None else sampling_steps
    t = torch.linspace(0, n_steps - 1, steps=s + 1)
    t = torch.cat((torch.tensor([-1]), t))
    return list(reversed(t.int().tolist()))
