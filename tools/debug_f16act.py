"""Debug: f16 U-Net eps with fp32 vs fp16 activation buffers (MPCD_UNET_F16_ACT), fused / unfused."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec
from tests._util import make_unet
d, H, C, B = 1, 32, 5, 24
net = make_unet(d, C, seed=d + H)
spec = NetSpec("unet", state_dim=d, horizon=H, context_dim=C, cfg=True, dtype="f16")
plan = DiffusionMPC(spec, net.state_dict(), variance_schedule="exponential", n_diffusion_steps=50)
g = torch.Generator().manual_seed(H)
x = torch.randn(B, H, d, generator=g)
ctx = torch.rand(1, C, generator=g) * 2 - 1
tt = torch.full((B,), 0, dtype=torch.long)
with torch.no_grad():
    ref = net(x, tt, ctx.expand(B, C), torch.zeros(B, 1))
for act in ("0", "1", "4", "8", "66", "48", "255"):
    for fuse in ("0",):
        os.environ["MPCD_UNET_F16_ACT"] = act
        os.environ["MPCD_UNET_FUSE"] = fuse
        ec, eu = plan.eps(x, 0, ctx)
        print(f"act={act} fuse={fuse}: max err {float((ec.cpu() - ref).abs().max()):.3e}", flush=True)
