"""Diagnostics: single noise-net forward on GPU vs oracle vs fp64."""
import sys, os, math
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec
from oracle import nets
B, H, d, C, N = 64, 16, 2, 4, 50
torch.manual_seed(0)
net = nets.ConditionedMLPNet(state_dim=d, horizon=H, context_dim=C).eval()
plan = DiffusionMPC(NetSpec("mlp", state_dim=d, horizon=H, context_dim=C), net.state_dict(), n_diffusion_steps=N)
ctx = torch.rand(1, C) * 2 - 1
x = torch.randn(B, H, d)
out = {}
for t in (49, 48, 25, 0):
    ec, eu = plan.eps(x, t, ctx)
    tt = torch.full((B,), t, dtype=torch.long)
    with torch.no_grad():
        rc = net(x, tt, ctx.expand(B, C), torch.zeros(B, 1))
        ru = net(x, tt, ctx.expand(B, C), torch.ones(B, 1))
    print(f"t={t}: cond max abs err {(ec.cpu() - rc).abs().max().item():.3e}  uncond {(eu.cpu() - ru).abs().max().item():.3e}")
    out[f"ec{t}"] = ec.cpu().numpy(); out[f"eu{t}"] = eu.cpu().numpy(); out[f"rc{t}"] = rc.numpy(); out[f"ru{t}"] = ru.numpy()
np.savez_compressed("gpurun_out/debug_eps.npz", x=x.numpy(), ctx=ctx.numpy(), **out)
