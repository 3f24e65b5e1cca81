"""Candidate-batch data parallelism: one process per GPU, RCCL over xGMI.

Each rank samples, rolls out and costs its own contiguous shard of candidates
(global index = rank * B_local + i; the Philox counter is keyed by that global index, so
results do not depend on the sharding). The one exchange per control step:
  1. all-gather of the per-candidate fp64 costs (B_local per rank)      -> every rank
  2. global argmin on every rank (NaN = +inf, lowest index on ties)     -> identical on all ranks
  3. broadcast of the winner's normalised [H, d] row from its owner     -> every rank
Two interchangeable implementations of that exchange:
  * select()/any_flag() below: torch.distributed collectives - any backend: "nccl" (= RCCL on ROCm)
    with device tensors, or "gloo" with CPU tensors (the CPU tests);
  * NativeComm: the communicator inside libmpcd.so (mpcd_comm_init, RCCL over xGMI) and mpcd_select,
    which keeps the whole exchange on the device - all-gather, argmin, and the winner's row handed to
    every rank by a sum all-reduce of (row if owner else zeros) - with no host round trip in between.
Weights, schedule and x0 are replicated, not exchanged.
"""
import ctypes

import torch
import torch.distributed as dist

from . import _native as N


def world(group=None):
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def shard(n_local, group=None):
    """(global_offset, total) of this rank's candidates under weak scaling (B_local per rank)."""
    rank, size = world(group)
    return rank * n_local, n_local * size


def _staged(t, group):
    """gloo moves host tensors only: device tensors of a gloo group go through a host copy."""
    return t.cpu() if t.is_cuda and dist.get_backend(group) == "gloo" else t


def gather_costs(cost_local, group=None):
    rank, size = world(group)
    if size == 1:
        return cost_local
    src = _staged(cost_local.contiguous(), group)
    out = torch.empty(size * src.numel(), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    return out.to(cost_local.device)


def argmin_nan_last(cost):
    """Host/CPU reference of the selection rule (used on gloo; the GPU path runs mpcd_argmin)."""
    c = torch.where(torch.isnan(cost), torch.full_like(cost, float("inf")), cost)
    best = torch.min(c)
    return int(torch.nonzero(c == best)[0, 0]), float(best)


def broadcast_row(row_local, owner, group=None):
    """row_local: this rank's candidate row if it owns the winner (any tensor of the right shape otherwise)."""
    rank, size = world(group)
    if size == 1:
        return row_local
    buf = _staged(row_local.contiguous(), group).clone()
    dist.broadcast(buf, src=dist.get_global_rank(group, owner) if group is not None else owner, group=group)
    return buf.to(row_local.device)


def any_flag(flag_local, group=None):
    """Max over ranks of a per-rank clip code (mpcd_clip_flag: 0 in range, 1 clip, 2 NaN seen), i.e. the
    global unnormalise clip rule across shards."""
    rank, size = world(group)
    if size == 1:
        return flag_local
    t = _staged(flag_local, group).clone()
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.to(flag_local.device)


def select(cost_local, rows_local, argmin, group=None):
    """The per-control-step exchange: all-gather costs, global argmin on every rank, broadcast the
    winner's row from its owner. cost_local [B_local] fp64, rows_local [B_local, ...];
    argmin(costs) -> (global index, cost). Returns (index, cost, row, all costs)."""
    rank, size = world(group)
    n_local = cost_local.shape[0]
    costs = gather_costs(cost_local, group)
    idx, best = argmin(costs)
    owner, local = divmod(idx, n_local)
    row = broadcast_row(rows_local[local if owner == rank else 0], owner, group)
    return idx, best, row, costs


class NativeComm:
    """Communicator owned by a planner's libmpcd context. Default: RCCL, one process per GPU; rank 0
    creates the 128-byte unique id, shipped to the other ranks over the torch.distributed group (any
    backend). Without an initialised process group (or with one rank) no communicator is made and the
    calls reduce to their single-rank forms inside the library.
    loopback=(nranks, rank, key): a virtual rank of an in-process loopback group instead (mpcd.h
    mpcd_comm_init_loopback): nranks planners on the same GPU, each driven by its own host thread,
    run the N-rank exchange through device copies - the single-GPU test of the RCCL code path."""

    def __init__(self, plan, group=None, loopback=None):
        self.plan, self.group = plan, group
        L = N.lib()
        if loopback is not None:
            self.size, self.rank, key = (int(v) for v in loopback)
            N.check(L.mpcd_comm_init_loopback(plan._ctx, self.size, self.rank, key), "mpcd_comm_init_loopback")
        else:
            self.rank, self.size = world(group)
        if self.size > 1 and loopback is None:
            uid = (ctypes.c_uint8 * N.MPCD_COMM_ID_BYTES)()
            if self.rank == 0:
                N.check(L.mpcd_comm_unique_id(uid), "mpcd_comm_unique_id")
            obj = [bytes(uid)]
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(obj, src=src, group=group)
            uid = (ctypes.c_uint8 * N.MPCD_COMM_ID_BYTES).from_buffer_copy(obj[0])
            N.check(L.mpcd_comm_init(plan._ctx, self.size, self.rank, uid), "mpcd_comm_init")
        nr, rk = ctypes.c_int32(), ctypes.c_int32()
        N.check(L.mpcd_comm_info(plan._ctx, ctypes.byref(nr), ctypes.byref(rk)), "mpcd_comm_info")
        assert (nr.value, rk.value) == ((self.size, self.rank) if self.size > 1 or loopback else (1, 0))
        self._best = torch.zeros(2, dtype=torch.float64, device=plan.device)

    def any_flag(self, flag_local):
        t = flag_local.clone()
        N.check(N.lib().mpcd_allreduce_max_i32(self.plan._ctx, ctypes.c_void_p(t.data_ptr()), t.numel(),
                                               self.plan._stream()), "mpcd_allreduce_max_i32")
        return t

    def select(self, cost_local, rows_local):
        """Same contract as select(): (global index, cost, winner row, all costs)."""
        n_local = cost_local.shape[0]
        row_shape = rows_local.shape[1:]
        row_len = rows_local[0].numel()
        costs = torch.empty(self.size * n_local, dtype=torch.float64, device=cost_local.device)
        row = torch.empty(row_len, dtype=torch.float32, device=cost_local.device)
        N.check(N.lib().mpcd_select(self.plan._ctx, ctypes.c_void_p(cost_local.contiguous().data_ptr()), n_local,
                                    ctypes.c_void_p(rows_local.contiguous().data_ptr()), row_len,
                                    ctypes.c_void_p(costs.data_ptr()), ctypes.c_void_p(self._best.data_ptr()),
                                    ctypes.c_void_p(row.data_ptr()), self.plan._stream()), "mpcd_select")
        host = self._best.cpu()
        return int(host.view(torch.int64)[1]), float(host[0]), row.view(row_shape), costs
