"""Host-side cost of one cfg2 control step's Python path (GPU box): plan.mpc_step with the library's mpcd_mpc_step
replaced by a no-op (everything else real: argument block, device tensors, ctypes), and its pieces timed alone.

  python tools/host_path.py"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, systems  # noqa: E402

cfg = bench.WORKLOADS["cfg2"]
torch.cuda.set_device(0)
spec = NetSpec("mlp", state_dim=cfg["d"], horizon=cfg["H"], context_dim=cfg["C"], dtype=cfg["dtype"])
plan = DiffusionMPC(spec, bench.synthetic_params(spec, seed=0), variance_schedule=cfg["schedule"], n_diffusion_steps=cfg["N"])
system = systems.get(cfg["system"])
x0s = np.random.default_rng(1).uniform(-1, 1, (400, system.n_x))
B = 4096
for i in range(5):
    plan.mpc_step(x0s[i], system, B, w=0.01, seed=2 + i)
torch.cuda.synchronize()


class NoStep:
    """the library with mpcd_mpc_step as a no-op returning MPCD_OK"""
    def __init__(self, lib):
        self._l = lib

    def __getattr__(self, n):
        if n == "mpcd_mpc_step":
            return lambda *a: 0
        return getattr(self._l, n)


def per_call(f, n=20000):
    for _ in range(200):
        f()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t0) / n * 1e6


real = plan._lib
plan._lib = NoStep(real)
us = per_call(lambda: plan.mpc_step(x0s[0], system, B, w=0.01, seed=3))
plan._lib = real
print(f"mpc_step Python path without the library call: {us:.2f} us")
fl = ctypes.c_int32()
print(f"  ctypes call (mpcd_last_step_flags):          {per_call(lambda: real.mpcd_last_step_flags(plan._ctx, ctypes.byref(fl))):.2f} us")
print(f"  torch.empty x2 on the device:                {per_call(lambda: (torch.empty((B, 32, 2), device=plan.device), torch.empty(B, dtype=torch.float64, device=plan.device))):.2f} us")
print(f"  plan._stream():                              {per_call(plan._stream):.2f} us")
print(f"  plan._system_desc(system):                   {per_call(lambda: plan._system_desc(system)):.2f} us")
print(f"  np.empty + ascontiguousarray:                {per_call(lambda: (np.empty((32, 2), dtype=np.float32), np.ascontiguousarray(x0s[0], dtype=np.float64))):.2f} us")
t0 = time.perf_counter()
for i in range(200):
    plan.mpc_step(x0s[i % 400], system, B, w=0.01, seed=2 + i)
torch.cuda.synchronize()
print(f"full mpc_step: {(time.perf_counter() - t0) / 200 * 1e3:.4f} ms; sampler kernel {plan.sample_ms_mean(200):.4f} ms")
