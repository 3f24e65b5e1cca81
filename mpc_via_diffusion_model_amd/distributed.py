"""Candidate-batch data parallelism: one process per GPU, RCCL over xGMI.

Each rank samples, rolls out and costs its own contiguous shard of candidates
(global index = rank * B_local + i; the Philox counter is keyed by that global index, so
results do not depend on the sharding). The one exchange per control step:
  1. all-gather of the per-candidate fp64 costs (B_local per rank)      -> every rank
  2. global argmin on every rank (NaN = +inf, lowest index on ties)     -> identical on all ranks
  3. broadcast of the winner's normalised [H, d] row from its owner     -> every rank
Works on any torch.distributed backend: "nccl" (= RCCL on ROCm) with device tensors, or "gloo"
with CPU tensors (the CPU tests). Weights, schedule and x0 are replicated, not exchanged.
"""
import torch
import torch.distributed as dist


def world(group=None):
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def shard(n_local, group=None):
    """(global_offset, total) of this rank's candidates under weak scaling (B_local per rank)."""
    rank, size = world(group)
    return rank * n_local, n_local * size


def gather_costs(cost_local, group=None):
    rank, size = world(group)
    if size == 1:
        return cost_local
    out = torch.empty(size * cost_local.numel(), dtype=cost_local.dtype, device=cost_local.device)
    dist.all_gather_into_tensor(out, cost_local.contiguous(), group=group)
    return out


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
    buf = row_local.contiguous().clone()
    dist.broadcast(buf, src=dist.get_global_rank(group, owner) if group is not None else owner, group=group)
    return buf


def any_flag(flag_local, group=None):
    """Logical OR of a per-rank int flag (the global unnormalise clip rule across shards)."""
    rank, size = world(group)
    if size == 1:
        return flag_local
    t = flag_local.clone()
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t


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
