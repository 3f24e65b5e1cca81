import sys, os, ctypes
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec
from mpc_via_diffusion_model_amd import _native as NN
from oracle import nets
B, H, d, C, N = 16, 16, 2, 4, 50
torch.manual_seed(0)
net = nets.ConditionedMLPNet(state_dim=d, horizon=H, context_dim=C).eval()
x = torch.randn(B, H, d)
ctx = torch.rand(1, C) * 2 - 1
plan = DiffusionMPC(NetSpec("mlp", state_dim=d, horizon=H, context_dim=C), net.state_dict(), n_diffusion_steps=N)
dbg = torch.zeros(14 * 32 * 256, device="cuda")
L = NN.lib()
L.mpcd_debug_set.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
L.mpcd_debug_set(plan._ctx, ctypes.c_void_p(dbg.data_ptr()))
ec, eu = plan.eps(x, 25, ctx)
torch.cuda.synchronize()
np.savez_compressed("gpurun_out/debug_layers.npz", dbg=dbg.cpu().numpy().reshape(14, 32, 256), x=x.numpy(),
                    ctx=ctx.numpy(), ec=ec.cpu().numpy(), eu=eu.cpu().numpy())
print("ok")
