"""Fresh-process helper for tests/test_gpu_threads.py: four host threads make the process's FIRST launches of
the MLP sampler, the rollout and the U-Net convs at the same moment (loopback communicator ranks for the MLP
step; independent U-Net planners), so the launch code's once-per-kernel attribute calls, the per-device CU
count and the occupancy cache are entered concurrently. Results must equal one planner run afterwards.
Exit code 0 and a final "OK" line on success."""
import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, systems  # noqa: E402
from mpc_via_diffusion_model_amd import distributed as D  # noqa: E402
from tests._util import make_mlp, make_unet  # noqa: E402


def run_threads(n, fn):
    out, errs = [None] * n, []
    gate = threading.Barrier(n)

    def body(r):
        try:
            torch.cuda.set_device(0)
            with torch.cuda.stream(torch.cuda.Stream()):
                gate.wait()
                out[r] = fn(r)
                torch.cuda.current_stream().synchronize()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    if any(t.is_alive() for t in ts):
        raise SystemExit("a thread hung")
    if errs:
        raise errs[0]
    return out


def main():
    n = 4
    sd = make_mlp(2, 32, 4, seed=3).state_dict()
    sysm = systems.double_int2d()
    x0 = np.array([0.3, -0.2, 0.1, 0.05])
    plans = [DiffusionMPC(NetSpec("mlp", 2, 32, 4, dtype="f32x3"), sd, n_diffusion_steps=25) for _ in range(n)]
    comms = [D.NativeComm(plans[r], loopback=(n, r, 4242)) for r in range(n)]
    res = run_threads(n, lambda r: plans[r].mpc_step(x0, sysm, 1024, seed=11, comm=comms[r]))
    full = DiffusionMPC(NetSpec("mlp", 2, 32, 4, dtype="f32x3"), sd, n_diffusion_steps=25)
    ref = full.mpc_step(x0, sysm, n * 1024, seed=11)
    for got in res:
        assert (got.best_index, got.best_cost) == (ref.best_index, ref.best_cost)
        np.testing.assert_array_equal(got.u_best, ref.u_best)

    usd = make_unet(4, 12, seed=5).state_dict()
    ctx = torch.rand(1, 12, generator=torch.Generator().manual_seed(1)) * 2 - 1
    uplans = [DiffusionMPC(NetSpec("unet", 4, 64, 12, dtype="f16"), usd, variance_schedule="cosine",
                           n_diffusion_steps=10) for _ in range(n)]
    outs = run_threads(n, lambda r: uplans[r].sample_trajectories(ctx, 2048, 64, seed=7).cpu())
    ref_u = uplans[0].sample_trajectories(ctx, 2048, 64, seed=7).cpu()
    for o in outs:
        assert torch.equal(o, ref_u)
    print("OK", flush=True)


if __name__ == "__main__":
    main()
