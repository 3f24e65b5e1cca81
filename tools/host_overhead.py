"""Host-side cost of one cfg2 control step (GPU box): wall time per plan.mpc_step against the GPU time of its
launches, and a cProfile of the Python around the libmpcd call.

  python tools/host_overhead.py [B]"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, systems  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cfg = bench.WORKLOADS["cfg2"]
torch.cuda.set_device(0)
spec = NetSpec("mlp", state_dim=cfg["d"], horizon=cfg["H"], context_dim=cfg["C"], dtype=cfg["dtype"])
plan = DiffusionMPC(spec, bench.synthetic_params(spec, seed=0), variance_schedule=cfg["schedule"], n_diffusion_steps=cfg["N"])
system = systems.get(cfg["system"])
x0s = np.random.default_rng(1).uniform(-1, 1, (400, system.n_x))


def step(i):
    return plan.mpc_step(x0s[i % 400], system, B, w=0.01, sample_fn="ddpm_cfg", seed=2 + i)


for i in range(20):
    step(i)
torch.cuda.synchronize()
n = 200
t0 = time.perf_counter()
ker = []
for i in range(n):
    step(i)
    ker.append(plan.last_sample_ms())
el = (time.perf_counter() - t0) / n
print(f"B={B}: {el * 1e3:.4f} ms per mpc_step, sampler kernel {np.mean(ker):.4f} ms, rest {el * 1e3 - np.mean(ker):.4f} ms")
pr = cProfile.Profile()
pr.enable()
for i in range(n):
    step(i)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(18)
