"""Diagnostics: per-step error profile of the MLP sampler vs the oracle (GPU)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec
from mpc_via_diffusion_model_amd import schedule as S
from oracle import nets, sampler, schedule

B, H, d, C, N = 64, 16, 2, 4, 50
torch.manual_seed(0)
net = nets.ConditionedMLPNet(state_dim=d, horizon=H, context_dim=C).eval()
plan = DiffusionMPC(NetSpec("mlp", state_dim=d, horizon=H, context_dim=C), net.state_dict(), n_diffusion_steps=N)
g = torch.Generator().manual_seed(3)
ctx = torch.rand(1, C, generator=g) * 2 - 1
noise = torch.randn(N + 1, B, H, d, generator=torch.Generator().manual_seed(11))
bufs = schedule.buffers("exponential", N)
ref = sampler.ddpm_cfg(net, bufs, ctx.expand(B, C), 0.01, B, H, noise=noise, return_chain=True).double()
got = plan.sample_trajectories(ctx, B, H, w=0.01, noise=noise, return_chain=True).cpu().double()
e = (got - ref).abs() / ref.abs().clamp_min(1)
print("per-step max elem err x1e5:", [round(e[s].max().item() * 1e5, 2) for s in range(N + 1)])
idx = np.unravel_index(e.argmax().item(), e.shape)
print("worst", idx, got[idx].item(), ref[idx].item())
# single-pair DDIM probe of eps: non-CFG MLP path, times [t, -1] -> x = x0 = a*x - b*eps
plan3 = DiffusionMPC(NetSpec("mlp", state_dim=d, horizon=H, context_dim=C, cfg=False), net.state_dict(),
                     n_diffusion_steps=N)
zeros = torch.zeros(B, 1)
x = noise[0]
for t in (0, 5, 25, 49):
    import ctypes
    from mpc_via_diffusion_model_amd import _native as Nn
    # run through sample_trajectories with an explicit 1-pair grid
    S.ddim_times_orig = S.ddim_times
    S.ddim_times = lambda n, s=None, t=t: [t, -1]
    out = plan3.sample_trajectories(ctx.expand(B, C), B, H, sample_fn="ddim", noise=noise[:2]).cpu().double()
    S.ddim_times = S.ddim_times_orig
    tt = torch.full((B,), t, dtype=torch.long)
    eps = net(x, tt, ctx.expand(B, C), zeros)
    a = bufs["sqrt_recip_alphas_cumprod"][t]; b = bufs["sqrt_recipm1_alphas_cumprod"][t]
    x0 = (a * x - b * eps).double()
    eps_gpu = (a.double() * x.double() - out) / b.double()
    print(f"t={t}: x0 max abs err {(out - x0).abs().max().item():.3e}; eps err max {(eps_gpu - eps.double()).abs().max().item():.3e} "
          f"(|eps| max {eps.abs().max().item():.2f})")
np.savez_compressed(os.path.join("gpurun_out", "debug_chain.npz"), got=got.numpy(), ref=ref.numpy(), noise=noise.numpy(),
                    ctx=ctx.numpy())
