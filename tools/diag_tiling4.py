"""Diagnostics (GPU) round 4: the alias-candidate nondeterminism under layout variants, and the U-Net
chain |x| maxima with Philox vs injected noise."""
import os
import sys

import torch

sys.path.insert(0, ".")
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, force_unet_tiling  # noqa: E402
from tests._util import make_unet  # noqa: E402


def absmax(B, N, philox, dtype="f32", sched="cosine"):
    d, H, C = 2, 16, 4
    net = make_unet(d, C, seed=6)
    plan = DiffusionMPC(NetSpec("unet", d, H, C, dtype=dtype), net.state_dict(), n_diffusion_steps=N,
                        variance_schedule=sched)
    ctx = torch.rand(1, C) * 2 - 1
    noise = None if philox else torch.randn(N + 1, B, H, d)
    am = torch.full((B,), -7.0, dtype=torch.float32, device="cuda")
    chain = plan.sample_trajectories(ctx, B, H, seed=3, noise=noise, return_chain=True, absmax_out=am)
    want = chain.abs().amax(dim=(0, 2, 3))
    bad = (am != want).nonzero().flatten()
    print(f"absmax B={B} N={N} philox={philox} {sched}: mismatches {bad.numel()} first {bad[:5].tolist()} "
          f"am {am[bad[:3]].tolist()} want {want[bad[:3]].tolist()}", flush=True)


def layer(B, lay, cand, env):
    d, H, C = 1, 32, 2
    net = make_unet(d, C, seed=7)
    plan = DiffusionMPC(NetSpec("unet", d, H, C, dtype="f32x3"), net.state_dict(), n_diffusion_steps=100)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(B, H, d, generator=g, device="cuda")
    ctx = torch.rand(1, C, generator=g, device="cuda") * 2 - 1
    for k in ("MPCD_UNET_NO_ALIAS", "MPCD_UNET_LDS_PAD"):
        os.environ.pop(k, None)
    os.environ.update(env)
    os.environ["MPCD_UNET_FORCE_BASE"] = "1"
    os.environ["MPCD_UNET_FORCE_LAYER"] = str(lay)
    force_unet_tiling(cand, -2)
    outs = [plan.eps(x, 33, ctx)[0].clone() for _ in range(4)]
    bad = [int((o != outs[0]).flatten(1).any(1).sum()) for o in outs[1:]]
    print(f"layer {lay} cand {cand} env {env}: repeat rows differing {bad}", flush=True)
    force_unet_tiling(-1, -1)


if __name__ == "__main__":
    for B in (3, 45):
        for philox in (True, False):
            for N in (1, 5):
                absmax(B, N, philox)
    absmax(45, 25, True, "f32x3", "exponential")
    for lay, cand in ((14, 2), (14, 4), (17, 4)):
        for env in ({}, {"MPCD_UNET_NO_ALIAS": "1"}, {"MPCD_UNET_LDS_PAD": "16384"}, {"MPCD_UNET_LDS_PAD": "65536"}):
            layer(2048, lay, cand, env)
