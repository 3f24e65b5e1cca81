"""Training-step throughput of the native trainer (csrc/train.hip): the cfg2-shaped MLP net (d=2, H=32, C=4) or
the cart-pole U-Net (--net unet: d=1, H=32, C=5), N=100; training samples per second over --steps timed steps
after --warmup, synthetic data and random-init weights."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_via_diffusion_model_amd import NetSpec  # noqa: E402
from mpc_via_diffusion_model_amd.training import DiffusionTrainer  # noqa: E402
from bench import synthetic_params  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=4096)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--net", default="mlp", choices=["mlp", "unet"])
a = ap.parse_args()
spec = NetSpec("mlp", 2, 32, 4) if a.net == "mlp" else NetSpec("unet", 1, 32, 5)
d, C = spec.state_dim, spec.context_dim
tr = DiffusionTrainer(spec, synthetic_params(spec, seed=0), n_diffusion_steps=100)
g = torch.Generator().manual_seed(0)
x0 = torch.rand(a.B, 32, d, generator=g) * 2 - 1
ctx = torch.rand(a.B, C, generator=g) * 2 - 1
draws = [tr.draw(a.B, (a.B, 32, d), generator=g) for _ in range(a.steps + a.warmup)]
for i in range(a.warmup):
    tr.train_step(x0, ctx, *draws[i])
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(a.steps):
    loss = tr.train_step(x0, ctx, *draws[a.warmup + i])
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(f"train {a.net} B={a.B}: {1e3 * el / a.steps:.2f} ms/step, {a.B * a.steps / el:.0f} samples/s, last loss {loss:.5f}")
