"""Denoising loops (oracle; test infrastructure only).

Restates, op for op (fp32 torch CPU):
  make_timesteps                      diffusion_model_base.py:25-27
  predict_start_from_noise / q_posterior   :127-147
  p_mean_variance_CFG                 :164-178   (x0 = (1+w)*x0_c - w*x0_u, clamp_(-1, 1))
  cart_pole_sample_loop               :181-209   (x_T = randn, one randn_like per step)
  ddpm_cart_pole_sample_fn            sample_functions.py:17-44 (t<0 -> 0, noise[t==0] = 0)
  run_CFG                             diffusion_model_base.py:394-418 (chain -> [S+1, B, H, d])
  ddim_sample                         :239-314   (eta = 0, grid linspace(0, N-1, N//5+1) + [-1])
``ddim_cfg`` is BUILD-DEFINED: the reference's ddim_sample cannot
drive the 4-arg CFG net, so CFG-DDIM has no reference output.

Noise: ``noise=None`` replays the reference's global-RNG stream (torch.randn then
randn_like per step); otherwise ``noise`` is a [S+1, B, H, d] tensor whose slice 0
is x_T and slice k the draw of step k (the injected-noise parity mode).
"""
import torch

from .schedule import buffers


def _take(table, t):
    # sample_functions.py:11-14 extract(): gather then broadcast over (H, d)
    return table.gather(-1, t).reshape(t.shape[0], 1, 1)


class _NoiseStream:
    def __init__(self, noise):
        self.noise = noise
        self.k = 0

    def draw(self, like):
        if self.noise is None:
            z = torch.randn(like.shape) if self.k == 0 else torch.randn_like(like)
        else:
            z = self.noise[self.k].clone()
        self.k += 1
        return z


def ddpm_cfg(net, bufs, context, w, batch, horizon, n_wo_noise=0, noise=None, return_chain=False):
    """run_CFG with sample_fn=ddpm_cart_pole_sample_fn. Returns [S+1,B,H,d] chain or final [B,H,d]."""
    n_steps = bufs["betas"].shape[0]
    shape = (batch, horizon, net.state_dim)
    rng = _NoiseStream(noise)
    with torch.no_grad():
        x = rng.draw(torch.empty(shape))
        chain = [x]
        for i in reversed(range(-n_wo_noise, n_steps)):
            t = torch.full((batch,), i, dtype=torch.long)
            if t[0] < 0:
                t = torch.zeros_like(t)
            unmasked = torch.zeros(context.size(0), 1)
            masked = torch.ones(context.size(0), 1)
            a, b = _take(bufs["sqrt_recip_alphas_cumprod"], t), _take(bufs["sqrt_recipm1_alphas_cumprod"], t)
            x0_c = a * x - b * net(x, t, context, unmasked)
            x0_u = a * x - b * net(x, t, context, masked)
            x0 = (1 + w) * x0_c - w * x0_u
            x0.clamp_(-1.0, 1.0)
            mean = _take(bufs["posterior_mean_coef1"], t) * x0 + _take(bufs["posterior_mean_coef2"], t) * x
            var = torch.exp(_take(bufs["posterior_log_variance_clipped"], t))
            z = rng.draw(x)
            z[t == 0] = 0
            x = mean + torch.sqrt(var) * z
            chain.append(x)
    if return_chain:
        return torch.stack(chain, dim=0)
    return x


def ddim_grid(n_steps, sampling_steps=None):
    """ddim_sample's time pairs (diffusion_model_base.py:251-259)."""
    s = n_steps // 5 if sampling_steps is None else sampling_steps
    times = torch.linspace(0, n_steps - 1, steps=s + 1)
    times = torch.cat((torch.tensor([-1]), times))
    times = list(reversed(times.int().tolist()))
    return list(zip(times[:-1], times[1:]))


def ddim(net, bufs, batch, horizon, context=None, noise=None, sampling_steps=None, return_chain=False):
    """Reference ddim_sample with a 3-arg net (TemporalUnet), hard_conds = {}."""
    n_steps = bufs["betas"].shape[0]
    shape = (batch, horizon, net.state_dim)
    rng = _NoiseStream(noise)
    eta = 0.0
    with torch.no_grad():
        x = rng.draw(torch.empty(shape))
        chain = [x]
        for tc, tn in ddim_grid(n_steps, sampling_steps):
            t = torch.full((batch,), tc, dtype=torch.long)
            t_next = torch.full((batch,), tn, dtype=torch.long)
            eps = net(x, t, context)
            x_start = _take(bufs["sqrt_recip_alphas_cumprod"], t) * x - _take(bufs["sqrt_recipm1_alphas_cumprod"], t) * eps
            if tn < 0:
                x = x_start
                chain.append(x)
                break
            alpha = _take(bufs["alphas_cumprod"], t)
            alpha_next = _take(bufs["alphas_cumprod"], t_next)
            sigma = eta * ((1 - alpha / alpha_next) * (1 - alpha_next) / (1 - alpha)).sqrt()
            c = (1 - alpha_next - sigma ** 2).sqrt()
            x = x_start * alpha_next.sqrt() + c * eps
            z = rng.draw(x)
            x = x + sigma * z
            chain.append(x)
    if return_chain:
        return torch.stack(chain, dim=0)
    return x


def ddim_cfg(net, bufs, context, w, batch, horizon, noise=None, sampling_steps=None, clamp_x0=False,
             return_chain=False):
    """BUILD-DEFINED CFG-DDIM: per pair
    x0 = (1+w)*x0_c - w*x0_u [optional clamp]; eps = (1+w)*eps_c - w*eps_u;
    x_next = x0*sqrt(abar_next) + sqrt(1-abar_next)*eps; the (0,-1) pair returns x0.
    One noise draw per pair is consumed (sigma = 0) as ddim_sample does."""
    n_steps = bufs["betas"].shape[0]
    shape = (batch, horizon, net.state_dim)
    rng = _NoiseStream(noise)
    with torch.no_grad():
        x = rng.draw(torch.empty(shape))
        chain = [x]
        for tc, tn in ddim_grid(n_steps, sampling_steps):
            t = torch.full((batch,), tc, dtype=torch.long)
            t_next = torch.full((batch,), tn, dtype=torch.long)
            unmasked = torch.zeros(context.size(0), 1)
            masked = torch.ones(context.size(0), 1)
            a, b = _take(bufs["sqrt_recip_alphas_cumprod"], t), _take(bufs["sqrt_recipm1_alphas_cumprod"], t)
            eps_c = net(x, t, context, unmasked)
            eps_u = net(x, t, context, masked)
            x0 = (1 + w) * (a * x - b * eps_c) - w * (a * x - b * eps_u)
            if clamp_x0:
                x0.clamp_(-1.0, 1.0)
            if tn < 0:
                x = x0
                chain.append(x)
                break
            eps = (1 + w) * eps_c - w * eps_u
            alpha_next = _take(bufs["alphas_cumprod"], t_next)
            c = (1 - alpha_next - 0.0 ** 2).sqrt()
            x = x0 * alpha_next.sqrt() + c * eps
            rng.draw(x)
            chain.append(x)
    if return_chain:
        return torch.stack(chain, dim=0)
    return x


def noise_slices_ddpm(n_steps, n_wo_noise):
    return n_steps + n_wo_noise + 1


def noise_slices_ddim(n_steps, sampling_steps=None):
    return len(ddim_grid(n_steps, sampling_steps)) + 1


__all__ = ["buffers", "ddpm_cfg", "ddim", "ddim_cfg", "ddim_grid", "noise_slices_ddpm", "noise_slices_ddim"]
