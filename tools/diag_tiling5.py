"""Diagnostics (GPU) round 5: alias-candidate nondeterminism vs occupancy / stream sync; differing rows."""
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
    for k in ("MPCD_UNET_NO_ALIAS", "MPCD_UNET_LDS_PAD", "MPCD_UNET_SYNC"):
        os.environ.pop(k, None)
    os.environ.update(env)
    os.environ["MPCD_UNET_FORCE_BASE"] = "1"
    os.environ["MPCD_UNET_FORCE_LAYER"] = str(lay)
    force_unet_tiling(cand, -2)
    outs = [torch.cat(plan.eps(x, 33, ctx), 0).clone() for _ in range(4)]
    rows = [(o != outs[0]).flatten(1).any(1).nonzero().flatten() for o in outs[1:]]
    mx = [float((o - outs[0]).abs().max()) for o in outs[1:]]
    print(f"layer {lay} cand {cand} env {env}: rows differing {[r.numel() for r in rows]} max {mx} "
          f"first {rows[0][:12].tolist()}", flush=True)
    force_unet_tiling(-1, -1)


for lay, cand in ((14, 2), (9, 0)):
    for env in ({}, {"MPCD_UNET_SYNC": "1"}, {"MPCD_UNET_LDS_PAD": "163840"}, {"MPCD_UNET_LDS_PAD": "40000"}):
        run(lay, cand, env)
