"""Diagnostics (GPU): the 16-row MLP x3 layout against the 32-row one (eps of both CFG branches) and
against the oracle, per candidate; MPCD_MLP_LAYOUT is read once per process, so each layout runs in a
child process."""
import os
import subprocess
import sys

import torch

sys.path.insert(0, ".")

if len(sys.argv) > 1:
    from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec
    from tests._util import make_mlp
    B, H, d, C = 8, 32, 2, 4
    net = make_mlp(d, H, C, seed=12)
    plan = DiffusionMPC(NetSpec("mlp", d, H, C, dtype="f32x3"), net.state_dict(), n_diffusion_steps=100)
    x = torch.randn(B, H, d, generator=torch.Generator().manual_seed(1))
    ctx = torch.rand(1, C, generator=torch.Generator().manual_seed(2)) * 2 - 1
    ec, eu = plan.eps(x, 37, ctx)
    tt = torch.full((B,), 37, dtype=torch.long)
    with torch.no_grad():
        rc = net(x, tt, ctx.expand(B, C), torch.zeros(B, 1))
        ru = net(x, tt, ctx.expand(B, C), torch.ones(B, 1))
    print("layout", os.environ.get("MPCD_MLP_LAYOUT"), "ec err per cand", [round(float(v), 6) for v in (ec.cpu() - rc).abs().flatten(1).max(1).values],
          "eu err per cand", [round(float(v), 6) for v in (eu.cpu() - ru).abs().flatten(1).max(1).values], flush=True)
    sys.exit(0)
for r in ("32x8", "16x8", "16x4"):
    subprocess.run([sys.executable, __file__, "x"], env=dict(os.environ, MPCD_MLP_LAYOUT=r), check=True)
