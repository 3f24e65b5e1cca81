"""Diagnostics (GPU): run-to-run determinism of every U-Net conv layer under each forced tiling at a
batch large enough for several workgroups per CU (MPCD_UNET_FORCE_LAYER applies the forced candidate
to one conv, the others take MPCD_UNET_FORCE_BASE), and the chain |x| maxima with a one-hot x_T.
This is how the packed-f32 Mish issue of the mx epilogue was localised (unet_mx.hip epilogue)."""
import os
import sys

import torch

sys.path.insert(0, ".")
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, force_unet_tiling  # noqa: E402
from tests._util import make_unet  # noqa: E402


def absmax_onehot():
    d, H, C, B, N = 2, 16, 4, 3, 1
    net = make_unet(d, C, seed=6)
    plan = DiffusionMPC(NetSpec("unet", d, H, C, dtype="f32"), net.state_dict(), n_diffusion_steps=N)
    ctx = torch.rand(1, C) * 2 - 1
    for q in range(8):
        noise = torch.full((N + 1, B, H, d), 0.1)
        noise[0].view(B, -1)[:, 4 * q:4 * q + 4] = 5.0
        am = torch.full((B,), -7.0, dtype=torch.float32, device="cuda")
        chain = plan.sample_trajectories(ctx, B, H, noise=noise, return_chain=True, absmax_out=am)
        print(f"one-hot quad {q}: am {am.tolist()} chain max {chain.abs().amax(dim=(0, 2, 3)).tolist()}", flush=True)


def layers(B, dtype):
    d, H, C = 1, 32, 2
    net = make_unet(d, C, seed=7)
    plan = DiffusionMPC(NetSpec("unet", d, H, C, dtype=dtype), net.state_dict(), n_diffusion_steps=100)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(B, H, d, generator=g, device="cuda")
    ctx = torch.rand(1, C, generator=g, device="cuda") * 2 - 1
    os.environ["MPCD_UNET_FORCE_BASE"] = "1"
    n_layers = 40
    for layer in range(n_layers):
        for cand in (0, 2, 4):
            os.environ["MPCD_UNET_FORCE_LAYER"] = str(layer)
            force_unet_tiling(cand, -2)
            outs = [plan.eps(x, 33, ctx)[0].clone() for _ in range(3)]
            bad = [int((o != outs[0]).flatten(1).any(1).sum()) for o in outs[1:]]
            print(f"{dtype} B={B} layer {layer} cand {cand}: repeat rows differing {bad}", flush=True)
    force_unet_tiling(-1, -1)


if __name__ == "__main__":
    absmax_onehot()
    layers(2048, "f32x3")
