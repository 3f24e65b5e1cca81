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


# ---- N virtual ranks on one GPU (mpcd_comm_init_loopback): the N-rank exchange code of mpcd_select /
# mpcd_mpc_step (rank offsets, gathered-cost order, owner-row sum all-reduce, flag max-reduction), each
# virtual rank a planner driven by its own host thread on its own HIP stream.

def _run_ranks(n, fn):
    """fn(rank) on n threads at once (a collective needs every rank inside the library together)."""
    import threading
    out, errs = [None] * n, []

    def body(r):
        try:
            torch.cuda.set_device(0)
            with torch.cuda.stream(torch.cuda.Stream()):
                out[r] = fn(r)
                torch.cuda.current_stream().synchronize()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a virtual rank hung"
    if errs:
        raise errs[0]
    return out


_KEY = [1000]


def _key():
    _KEY[0] += 1
    return _KEY[0]


@pytest.mark.parametrize("nranks,b_local,clip_rule", [(2, 512, "chain"), (3, 200, "chain"), (2, 300, "final"),
                                                      (4, 64, "chain")])
def test_loopback_mpc_step_equals_single_process(nranks, b_local, clip_rule):
    """mpcd_mpc_step with an nranks loopback communicator on every virtual rank == one planner over the
    whole batch: same global winner, cost, trajectory and all-gathered costs (Philox keyed by the global
    candidate index, so the shards draw the batch's numbers)."""
    net = make_mlp(2, 32, 4, seed=3)
    sd = net.state_dict()
    sysm = systems.double_int2d()
    x0 = np.array([0.3, -0.2, 0.1, 0.05])
    key = _key()
    plans = [DiffusionMPC(NetSpec("mlp", 2, 32, 4, dtype="f32x3"), sd, n_diffusion_steps=25) for _ in range(nranks)]
    comms = [D.NativeComm(plans[r], loopback=(nranks, r, key)) for r in range(nranks)]
    res = _run_ranks(nranks, lambda r: [plans[r].mpc_step(x0, sysm, b_local, seed=11, comm=comms[r], clip_rule=clip_rule)
                                        for _ in range(2)])  # two steps: the group is reusable
    full = DiffusionMPC(NetSpec("mlp", 2, 32, 4, dtype="f32x3"), sd, n_diffusion_steps=25)
    ref = full.mpc_step(x0, sysm, nranks * b_local, seed=11, clip_rule=clip_rule)
    for r in range(nranks):
        for got in res[r]:
            assert (got.best_index, got.best_cost) == (ref.best_index, ref.best_cost)
            np.testing.assert_array_equal(got.u_best, ref.u_best)
            assert torch.equal(got.costs.cpu(), ref.costs.cpu())
            assert torch.equal(got.u_norm, ref.u_norm[r * b_local:(r + 1) * b_local])
    # the composed step (mpcd_select + flag max over the loopback group) agrees too
    res2 = _run_ranks(nranks, lambda r: plans[r].mpc_step(x0, sysm, b_local, seed=11, comm=comms[r], native=False,
                                                          clip_rule=clip_rule))
    for got in res2:
        assert (got.best_index, got.best_cost) == (ref.best_index, ref.best_cost)
        np.testing.assert_array_equal(got.u_best, ref.u_best)


def test_loopback_select_winner_on_rank1_nan_and_ties():
    """Crafted per-rank costs: the winner is owned by rank 1; NaNs on every rank rank as +inf; an exact tie
    between ranks 1 and 2 resolves to the lower global index; the winner's row reaches every rank; clip
    codes max-reduce (a NaN code 2 on one rank beats a clip 1 on another)."""
    n, b = 3, 5
    plans = [_plan() for _ in range(n)]
    key = _key()
    comms = [D.NativeComm(plans[r], loopback=(n, r, key)) for r in range(n)]
    costs = [[4.0, float("nan"), 3.0, 9.0, 8.0],
             [7.0, 5.0, 1.5, float("nan"), 2.0],
             [1.5, float("nan"), 6.0, 1.5, 3.0]]
    flags = [[0, 1], [1, 0], [0, 2]]

    def body(r):
        cost = torch.tensor(costs[r], dtype=torch.float64, device="cuda")
        rows = (torch.arange(b * 6, dtype=torch.float32, device="cuda") + 100 * r).view(b, 3, 2)
        idx, best, row, allc = comms[r].select(cost, rows)
        fl = comms[r].any_flag(torch.tensor(flags[r], dtype=torch.int32, device="cuda"))
        return idx, best, row.cpu(), allc.cpu(), fl.cpu().tolist()

    out = _run_ranks(n, body)
    want_row = (torch.arange(b * 6, dtype=torch.float32) + 100).view(b, 3, 2)[2]
    flat = torch.tensor(sum(costs, []), dtype=torch.float64)
    for idx, best, row, allc, fl in out:
        assert (idx, best) == (1 * b + 2, 1.5)  # rank 1, local 2 (ties with global 10 and 13)
        assert torch.equal(row, want_row)
        assert torch.equal(allc.isnan(), flat.isnan()) and torch.equal(allc[~flat.isnan()], flat[~flat.isnan()])
        assert fl == [1, 2]
