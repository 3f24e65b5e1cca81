"""The multi-process data-parallel step on the one GPU this box has (the 8-GPU curve is the
driver's): two fresh child processes on cuda:0 form a world-size-2 gloo group, each runs mpc_step on its half
of the BASELINE cfg2 candidates (2 x 2,048; global candidate index = rank * 2,048 + i keys the Philox draws),
the exchange (all-gather of the fp64 costs, global argmin, winner row from its owner) goes through
torch.distributed, and both ranks must return exactly the single-process winner, cost, row and cost vector of
one 4,096-candidate mpc_step. Each child also runs NativeComm's unique-id hand-off (mpcd_comm_unique_id on
rank 0, broadcast over the group); the RCCL init itself needs one GPU per rank and stays with the driver's
multi-GPU run."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, systems

from ._util import make_mlp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(tmp_path, world, b_total, mode, timeout=200):
    port, out = str(_free_port()), str(tmp_path / "mp")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_mp_mpc_step_worker.py"), str(r), str(world), port,
                               out, str(b_total), mode], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=timeout)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return procs, logs, out


def _reference(b_total):
    H, d, C = 32, 2, 4
    net = make_mlp(d, H, C, seed=0)
    plan = DiffusionMPC(NetSpec("mlp", state_dim=d, horizon=H, context_dim=C, dtype="f32x3"), net.state_dict(),
                        variance_schedule="exponential", n_diffusion_steps=100)
    x0 = np.random.default_rng(1).uniform(-1, 1, C)
    ref = plan.mpc_step(x0, systems.get("double_int2d"), b_total, w=0.01, seed=2)
    torch.cuda.synchronize()
    return ref, ref.costs.cpu().numpy()


@pytest.mark.timeout(240)
def test_two_processes_on_one_gpu_match_one_process(tmp_path):
    world, b_total = 2, 4096
    procs, logs, out = _run_ranks(tmp_path, world, b_total, "gloo")
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r][-3000:]}"
    ref, ref_costs = _reference(b_total)
    uids = []
    for r in range(world):
        z = np.load(f"{out}.rank{r}.npz")
        np.testing.assert_array_equal(z["costs"], ref_costs)  # all-gather in global index order, same bits
        assert int(z["best_index"]) == ref.best_index and float(z["best_cost"]) == ref.best_cost, r
        np.testing.assert_array_equal(z["u_best"], ref.u_best)
        np.testing.assert_array_equal(z["u0"], ref.u0)
        uids.append(z["uid"])
    assert uids[0].any() and all(np.array_equal(u, uids[0]) for u in uids), "NativeComm unique id not shared"
    print(f"2 processes x {b_total // world} candidates on cuda:0 = one process x {b_total}: winner {ref.best_index}, "
          f"cost {ref.best_cost:.6f}")


@pytest.mark.timeout(240)
def test_two_processes_rccl_exchange_on_one_gpu(tmp_path):
    """The product exchange (NativeComm: RCCL communicator inside libmpcd.so, native mpcd_mpc_step) with two ranks on
    the one device this box has. RCCL may refuse a communicator with two ranks on one GPU: then this is skipped and the
    driver's multi-GPU run is the first RCCL run with more than one rank."""
    world, b_total = 2, 4096
    procs, logs, out = _run_ranks(tmp_path, world, b_total, "rccl", timeout=150)
    if any(p.returncode == 3 for p in procs):
        msg = next(ln for lg in logs for ln in lg.splitlines() if "RCCL_INIT_REFUSED" in ln)
        pytest.skip(f"RCCL refuses two ranks on one device: {msg[:300]}")
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r][-3000:]}"
    ref, ref_costs = _reference(b_total)
    for r in range(world):
        z = np.load(f"{out}.rank{r}.npz")
        np.testing.assert_array_equal(z["costs"], ref_costs)
        assert int(z["best_index"]) == ref.best_index and float(z["best_cost"]) == ref.best_cost, r
        np.testing.assert_array_equal(z["u_best"], ref.u_best)
    print(f"RCCL, 2 ranks on cuda:0: winner {ref.best_index} = one process")
