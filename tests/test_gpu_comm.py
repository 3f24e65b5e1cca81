"""GPU: the C-ABI exchange (mpcd_select / RCCL communicator in libmpcd.so) against the torch path.

One GPU here: the communicator is a real one-rank RCCL communicator (mpcd_comm_init with nranks = 1),
so every collective runs through RCCL; the N > 1 logic (owner-or-zeros row + sum all-reduce, rank
offsets) is the same code, and the torch.distributed form of the exchange is covered at world size 2
on CPU (tests/test_distributed.py)."""
import ctypes

import numpy as np
import pytest
import torch

from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, systems
from mpc_via_diffusion_model_amd import _native as N
from mpc_via_diffusion_model_amd import distributed as D

from ._util import make_mlp

pytestmark = pytest.mark.gpu


def _plan():
    net = make_mlp(2, 32, 4, seed=3)
    return DiffusionMPC(NetSpec("mlp", 2, 32, 4), net.state_dict(), n_diffusion_steps=25)


def _rccl_one_rank(plan):
    L = N.lib()
    uid = (ctypes.c_uint8 * N.MPCD_COMM_ID_BYTES)()
    N.check(L.mpcd_comm_unique_id(uid), "mpcd_comm_unique_id")
    N.check(L.mpcd_comm_init(plan._ctx, 1, 0, uid), "mpcd_comm_init")
    nr, rk = ctypes.c_int32(), ctypes.c_int32()
    N.check(L.mpcd_comm_info(plan._ctx, ctypes.byref(nr), ctypes.byref(rk)), "mpcd_comm_info")
    assert (nr.value, rk.value) == (1, 0)
    assert L.mpcd_comm_init(plan._ctx, 1, 0, uid) == -3  # once per context


@pytest.mark.parametrize("rccl", [False, True])
def test_native_select_matches_torch_exchange(rccl):
    plan = _plan()
    if rccl:
        _rccl_one_rank(plan)
    comm = D.NativeComm(plan)
    sysm = systems.double_int2d()
    x0 = np.array([0.3, -0.2, 0.1, 0.05])
    a = plan.mpc_step(x0, sysm, 512, seed=11, native=False)           # torch exchange, composed step
    b = plan.mpc_step(x0, sysm, 512, seed=11, comm=comm, native=False)  # mpcd_select, composed step
    c = plan.mpc_step(x0, sysm, 512, seed=11, comm=comm)                # mpcd_mpc_step (RCCL branch if rccl)
    for r in (b, c):
        assert (a.best_index, a.best_cost) == (r.best_index, r.best_cost)
        np.testing.assert_array_equal(a.u_best, r.u_best)
        assert torch.equal(a.costs, r.costs)


def test_native_select_nan_and_ties():
    plan = _plan()
    _rccl_one_rank(plan)
    comm = D.NativeComm(plan)
    cost = torch.tensor([3.0, float("nan"), 1.0, 1.0, 2.0], dtype=torch.float64, device="cuda")
    rows = torch.arange(5 * 6, dtype=torch.float32, device="cuda").view(5, 3, 2)
    idx, best, row, costs = comm.select(cost, rows)
    assert (idx, best) == (2, 1.0)
    assert torch.equal(row, rows[2]) and torch.equal(costs.isnan(), cost.isnan())
    flag = comm.any_flag(torch.tensor([0, 1], dtype=torch.int32, device="cuda"))
    assert flag.tolist() == [0, 1]
    buf = torch.arange(4, dtype=torch.float32, device="cuda")
    N.check(N.lib().mpcd_broadcast_f32(plan._ctx, ctypes.c_void_p(buf.data_ptr()), 4, 0, plan._stream()), "bcast")
    g = torch.empty(4, dtype=torch.float32, device="cuda")
    N.check(N.lib().mpcd_allgather_f32(plan._ctx, ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(g.data_ptr()), 4,
                                       plan._stream()), "allgather")
    assert torch.equal(g, buf)
