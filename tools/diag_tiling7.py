"""Diagnostics (GPU) round 7: the co-resident GN-layer nondeterminism with a variant library (MPCD_LIB)."""
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
print("lib", os.environ.get("MPCD_LIB"))
for lay, cand in ((14, 2), (9, 0), (-1, 0), (-1, 2)):
    os.environ["MPCD_UNET_FORCE_BASE"] = "1" if lay >= 0 else str(cand)
    os.environ["MPCD_UNET_FORCE_LAYER"] = str(lay)
    force_unet_tiling(cand, -2)
    outs = [torch.cat(plan.eps(x, 33, ctx), 0).clone() for _ in range(4)]
    rows = [(o != outs[0]).flatten(1).any(1).nonzero().flatten() for o in outs[1:]]
    print(f"layer {lay} cand {cand}: rows differing {[r.numel() for r in rows]}", flush=True)
force_unet_tiling(-1, -1)
