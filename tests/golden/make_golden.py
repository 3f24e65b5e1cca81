"""Regenerate the golden fixtures from the oracle (which is pinned by the reference KATs in
tests/test_oracle_kats.py). Weights are not stored: they are the oracle module's default init under
torch.manual_seed(seed), and each fixture records the SHA-256 of the resulting parameter blob so a
changed initialiser is caught instead of silently producing new numbers.

    python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import nets, normalizer, sampler, schedule  # noqa: E402
from oracle import systems as osys  # noqa: E402


def blob_sha(module):
    h = hashlib.sha256()
    for v in module.state_dict().values():
        h.update(v.detach().contiguous().numpy().tobytes())
    return h.hexdigest()


def mlp(seed, d, H, C):
    torch.manual_seed(seed)
    return nets.ConditionedMLPNet(state_dim=d, horizon=H, context_dim=C).eval()


def unet(seed, d, C, mults=(1, 2, 4)):
    torch.manual_seed(seed)
    return nets.ConditionedTemporalUnet(state_dim=d, context_dim=C, dim_mults=mults).eval()


CASES = {
    # BASELINE cfg 1 shape: MLP, H=16, d=2, C=4, N=50 CFG-DDPM, double integrator cost + argmin
    "mlp_cfg1_ddpm": dict(net="mlp", seed=0, d=2, H=16, C=4, N=50, B=16, sampler="ddpm_cfg", nwo=0,
                          schedule="exponential", system="double_int2d"),
    # CFG-DDIM (build-defined), reference grid N//5, clamp on
    "mlp_ddim_cfg": dict(net="mlp", seed=1, d=2, H=32, C=4, N=100, B=16, sampler="ddim_cfg", clamp=True,
                         schedule="exponential", system="double_int2d"),
    # cart-pole U-Net (cfg 4 family at oracle size): d=1, C=5, H=32, N=25, nwo=5, calMPCCost
    "unet_cartpole_ddpm": dict(net="unet", seed=2, d=1, H=32, C=5, N=25, B=4, sampler="ddpm_cfg", nwo=5,
                               schedule="exponential", system="cartpole_lin5"),
}


def make(name, c):
    net = mlp(c["seed"], c["d"], c["H"], c["C"]) if c["net"] == "mlp" else unet(c["seed"], c["d"], c["C"])
    bufs = schedule.buffers(c["schedule"], c["N"])
    g = torch.Generator().manual_seed(100 + c["seed"])
    B, H, d, C = c["B"], c["H"], c["d"], c["C"]
    nx = osys.system_info(c["system"])["nx"]
    x0 = torch.rand(nx, generator=g, dtype=torch.float64) * 2 - 1
    lim = torch.ones(C)
    ctx = normalizer.normalize(x0[:C][None], -lim, lim).float() if nx >= C else torch.rand(1, C, generator=g) * 2 - 1
    if c["sampler"] == "ddpm_cfg":
        S = c["N"] + c.get("nwo", 0)
        noise = torch.randn(S + 1, B, H, d, generator=g)
        chain = sampler.ddpm_cfg(net, bufs, ctx.expand(B, C), 0.01, B, H, c.get("nwo", 0), noise=noise,
                                 return_chain=True)
    else:
        S = len(sampler.ddim_grid(c["N"]))
        noise = torch.randn(S + 1, B, H, d, generator=g)
        chain = sampler.ddim_cfg(net, bufs, ctx.expand(B, C), 0.01, B, H, noise=noise, clamp_x0=c.get("clamp", False),
                                 return_chain=True)
    u = normalizer.unnormalize(chain[-1], -torch.ones(d), torch.ones(d))
    cost = osys.rollout_cost(c["system"], x0.numpy(), u.double().numpy())
    np.savez_compressed(os.path.join(HERE, name + ".npz"), weights_sha256=np.array(blob_sha(net)),
                        noise=noise.numpy(), context=ctx.numpy(), x0=x0.numpy(), chain=chain.numpy(),
                        cost=cost, best=np.array(osys.argmin(cost)))


if __name__ == "__main__":
    for k, v in CASES.items():
        make(k, v)
        print("wrote", k, os.path.getsize(os.path.join(HERE, k + ".npz")), "bytes")
