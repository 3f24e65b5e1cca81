"""Diagnostics (GPU) round 6: LDS guard padding vs workgroups per CU for the nondeterministic tilings."""
import os
import sys

import torch

sys.path.insert(0, ".")
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, force_unet_tiling  # noqa: E402
from tests._util import make_unet  # noqa: E402

d, H, C, B = 1, 32, 2, 2048
net = make_unet(d, C, seed=7)
plan = DiffusionMPC(NetSpec("unet", d, H, C, dtype="f32x3"), net.state_dict(), n_diffusion_steps=100)
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.randn(B, H, d, generator=g, device="cuda")
ctx = torch.rand(1, C, generator=g, device="cuda") * 2 - 1


def run(lay, cand, env):
    for k in ("MPCD_UNET_NO_ALIAS", "MPCD_UNET_LDS_PAD", "MPCD_UNET_SYNC", "MPCD_UNET_LDS_FRONT"):
        os.environ.pop(k, None)
    os.environ.update(env)
    os.environ["MPCD_UNET_FORCE_BASE"] = "1"
    os.environ["MPCD_UNET_FORCE_LAYER"] = str(lay)
    force_unet_tiling(cand, -2)
    outs = [torch.cat(plan.eps(x, 33, ctx), 0).clone() for _ in range(4)]
    rows = [(o != outs[0]).flatten(1).any(1).nonzero().flatten() for o in outs[1:]]
    print(f"layer {lay} cand {cand} env {env}: rows differing {[r.numel() for r in rows]}", flush=True)
    force_unet_tiling(-1, -1)


# layer 14 cand 2: lds 42256 (3 per CU); layer 9 cand 0: lds 72208 (2 per CU)
for pad in ():
    run(14, 2, {"MPCD_UNET_LDS_PAD": str(pad)})
for pad in ():
    run(9, 0, {"MPCD_UNET_LDS_PAD": str(pad)})
for fr in (0, 1024, 8192):
    run(14, 2, {"MPCD_UNET_LDS_FRONT": str(fr)})
    run(9, 0, {"MPCD_UNET_LDS_FRONT": str(fr)})
