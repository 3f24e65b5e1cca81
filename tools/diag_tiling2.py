"""Diagnostics (GPU) round 2: U-Net chain |x| maxima vs N, and determinism per forced tiling at large B."""
import sys

import torch

sys.path.insert(0, ".")
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, force_unet_tiling  # noqa: E402
from tests._util import make_unet  # noqa: E402


def absmax_diag(N, dtype):
    d, H, C, B = 2, 16, 4, 45
    net = make_unet(d, C, seed=6)
    plan = DiffusionMPC(NetSpec("unet", d, H, C, dtype=dtype), net.state_dict(), n_diffusion_steps=N,
                        variance_schedule="cosine")
    ctx = torch.rand(1, C) * 2 - 1
    am = torch.full((B,), -7.0, dtype=torch.float32, device="cuda")
    chain = plan.sample_trajectories(ctx, B, H, seed=3, return_chain=True, absmax_out=am)
    per = chain.abs().amax(dim=(2, 3))
    print(f"N={N} {dtype}: all-slice match {int((per.amax(0) == am).sum())}/{B}; am[:4]={am[:4].tolist()}")
    print("   per-slice maxima cand 0:", [round(float(v), 4) for v in per[:, 0]])


def det_diag(d, H, C, B, dtype):
    net = make_unet(d, C, seed=7)
    plan = DiffusionMPC(NetSpec("unet", d, H, C, dtype=dtype), net.state_dict(), n_diffusion_steps=100)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(B, H, d, generator=g, device="cuda")
    ctx = torch.rand(1, C, generator=g, device="cuda") * 2 - 1
    outs = []
    for i in list(range(12)) + [-1]:
        force_unet_tiling(i, -2)
        a = plan.eps(x, 33, ctx)[0].clone()
        b = plan.eps(x, 33, ctx)[0].clone()
        rows = (a != b).flatten(1).any(1).nonzero().flatten()
        print(f"{dtype} B={B} cand {i}: self-repeat rows differing {rows.numel()} first {rows[:8].tolist()}")
        outs.append(a)
    force_unet_tiling(-1, -1)
    for i in range(1, len(outs)):
        rows = (outs[i] != outs[0]).flatten(1).any(1).nonzero().flatten()
        print(f"   cand {i} vs cand 0: rows differing {rows.numel()} first {rows[:8].tolist()}")


if __name__ == "__main__":
    for N in (1, 2, 5):
        for dt in ("f32", "f32x3"):
            absmax_diag(N, dt)
    det_diag(1, 32, 2, 16384, "f32")
    det_diag(1, 32, 2, 16384, "f32x3")
    det_diag(1, 32, 2, 2048, "f32x3")
