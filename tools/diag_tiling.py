"""Diagnostics (GPU): chain |x| maxima of the U-Net sampler per slice, and per-candidate eps differences
of forced U-Net tilings against the measured pick."""
import sys

import torch

sys.path.insert(0, ".")
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, force_unet_tiling  # noqa: E402
from tests._util import make_unet  # noqa: E402


def absmax_diag():
    d, H, C, N, B = 2, 16, 4, 25, 45
    net = make_unet(d, C, seed=6)
    plan = DiffusionMPC(NetSpec("unet", d, H, C, dtype="f32x3"), net.state_dict(), n_diffusion_steps=N)
    ctx = torch.rand(1, C) * 2 - 1
    am = torch.empty(B, dtype=torch.float32, device="cuda")
    chain = plan.sample_trajectories(ctx, B, H, seed=3, return_chain=True, absmax_out=am)
    per = chain.abs().amax(dim=(2, 3))  # [S+1, B]
    for k in range(per.shape[0]):
        print("from slice", k, "match", int((per[k:].amax(0) == am).sum()), "of", B)
    am2 = torch.empty(B, dtype=torch.float32, device="cuda")
    chain2 = plan.sample_trajectories(ctx, B, H, seed=3, return_chain=True, absmax_out=am2)
    print("second call equal chain", torch.equal(chain, chain2), "absmax match", int((per.amax(0) == am2).sum()))


def tiling_diag(d, H, C, B, dtype):
    net = make_unet(d, C, seed=7)
    plan = DiffusionMPC(NetSpec("unet", d, H, C, dtype=dtype), net.state_dict(), n_diffusion_steps=100)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(B, H, d, generator=g, device="cuda")
    ctx = torch.rand(1, C, generator=g, device="cuda") * 2 - 1
    force_unet_tiling(-1, -1)
    rc, ru = plan.eps(x, 33, ctx)
    rc2, ru2 = plan.eps(x, 33, ctx)
    print(f"{dtype} d={d} H={H} B={B}: repeat equal {torch.equal(rc, rc2) and torch.equal(ru, ru2)}")
    for i in range(12):
        force_unet_tiling(i, -2)
        ec, eu = plan.eps(x, 33, ctx)
        dc = float((ec - rc).abs().max())
        du = float((eu - ru).abs().max())
        nbad = int(((ec != rc).flatten(1).any(1)).sum())
        print(f"  conv cand {i}: max diff cond {dc:.3e} uncond {du:.3e} rows differing {nbad}")
    for j in range(6):
        force_unet_tiling(-1, j)
        ec, eu = plan.eps(x, 33, ctx)
        print(f"  block cand {j}: max diff {float((ec - rc).abs().max()):.3e} {float((eu - ru).abs().max()):.3e}")
    force_unet_tiling(-2 + 1, -2)
    ec, eu = plan.eps(x, 33, ctx)
    print(f"  measured convs, unfused blocks: {float((ec - rc).abs().max()):.3e}")
    force_unet_tiling(-1, -1)


if __name__ == "__main__":
    absmax_diag()
    for args in [(1, 32, 2, 64, "f32x3"), (1, 32, 2, 16384, "f32x3"), (4, 64, 12, 64, "f16"), (4, 64, 12, 8192, "f16")]:
        tiling_diag(*args)
