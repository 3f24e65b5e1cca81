"""Per-layer shader-clock breakdown of the MLP sampler (experiment build -DMPCD_PROF_LAYERS).

  python -m mpc_via_diffusion_model_amd.build prof MPCD_PROF_LAYERS      # here
  MPCD_LIB=mpc_via_diffusion_model_amd/libmpcd_prof.so python tools/layer_prof.py   # GPU box
Prints cycles per step (work / barrier wait) for each segment, averaged over 32 waves of 8 WGs."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec  # noqa: E402
from mpc_via_diffusion_model_amd import _native  # noqa: E402
from oracle import nets  # noqa: E402

torch.manual_seed(0)
net = nets.ConditionedMLPNet(state_dim=2, horizon=32, context_dim=4)
plan = DiffusionMPC(NetSpec("mlp", state_dim=2, horizon=32, context_dim=4, dtype=os.environ.get("DTYPE", "f32")), net.state_dict(),
                    variance_schedule="exponential", n_diffusion_steps=100)
ctx = torch.rand(1, 4) * 2 - 1
B = int(os.environ.get("B", 4096))
plan.sample_trajectories(ctx, B, 32, seed=1)
dbg = torch.zeros(14 * 32 * 256, device="cuda")
L = _native.lib()
L.mpcd_debug_set.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
L.mpcd_debug_set(plan._ctx, ctypes.c_void_p(dbg.data_ptr()))
plan.sample_trajectories(ctx, B, 32, seed=1)
torch.cuda.synchronize()
print(f"kernel ms {plan.last_sample_ms():.3f}")
ck = dbg[8 * 4 * 32: 8 * 4 * 32 + 16].cpu().numpy().reshape(8, 2)
se = dbg[4096: 4096 + 2 * 1024].cpu().view(torch.int32).numpy().astype(np.int64).reshape(-1, 2)
se = se[se[:, 1] != 0]
nb = len(se)
base = se[:, 0].min()
st, en = (se[:, 0] - base) / 100.0, (se[:, 1] - base) / 100.0  # microseconds
print(f"blocks {nb}: loop start us min/med/max {st.min():.1f}/{np.median(st):.1f}/{st.max():.1f}; "
      f"end min/med/max {en.min():.1f}/{np.median(en):.1f}/{en.max():.1f}")
print("slowest blocks (id, start, end):", [(int(i), round(float(st[i]), 1), round(float(en[i]), 1)) for i in np.argsort(-en)[:6]])
print(f"shader clock {float(np.median(ck[:, 0] / ck[:, 1])) * 0.1:.3f} GHz (memtime / memrealtime, 8 blocks)")
t = dbg[: 32 * 32].cpu().numpy().reshape(32, 32) / 100.0
# segment k accumulates the barrier-to-barrier spans that end at the k-th barrier of a step; the staging barrier
# before the loop takes index 0, so a step's first span (the cond tables + Linear 0) lands in index 1 and its last
# (the final Linear + update) in index 0
names = (["final+upd", "tbl+L0"] + [f"L{l}" for l in range(1, 13)] + ["-", "tail"] if os.environ.get("H2") else
         ["final+w1"] + [f"L{l}" for l in range(13)] + ["-", "tail"])
tot = t.sum(1).mean()
print(f"cycles/step per wave: {tot:.0f}")
for k in range(16):
    w, b = t[:, 2 * k].mean(), t[:, 2 * k + 1].mean()
    print(f"{names[k]:>9}: work {w:8.0f}  wait {b:8.0f}   (work max {t[:, 2 * k].max():8.0f})")
