"""Candidate-batch data parallelism on CPU (gloo, world size 2): each rank samples + costs its
shard with the oracle, then mpc_step's exchange (distributed.select) must pick the same winner,
cost and row as one process over the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mpc_via_diffusion_model_amd import distributed as D
from oracle import nets, normalizer, sampler, schedule
from oracle import systems as osys

B_LOCAL, H, d, C, N = 24, 16, 2, 4, 25


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pipeline(world):
    torch.manual_seed(0)
    net = nets.ConditionedMLPNet(state_dim=d, horizon=H, context_dim=C).eval()
    x0 = np.array([0.2, -0.4, 0.1, 0.3])
    one = torch.ones(C)
    ctx = normalizer.normalize(torch.from_numpy(x0)[None], -one, one).float()
    noise = torch.randn(N + 1, B_LOCAL * world, H, d, generator=torch.Generator().manual_seed(5))
    return net, x0, ctx, noise


def _shard_costs(net, x0, ctx, noise, lo, hi):
    x = sampler.ddpm_cfg(net, schedule.buffers("exponential", N), ctx.expand(hi - lo, C), 0.01, hi - lo, H,
                         noise=noise[:, lo:hi].contiguous())
    u = normalizer.unnormalize(x, -torch.ones(d), torch.ones(d))
    return torch.from_numpy(osys.rollout_cost("double_int2d", x0, u.double().numpy())), x


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net, x0, ctx, noise = _pipeline(world)
        off, total = D.shard(B_LOCAL)
        assert (off, total) == (rank * B_LOCAL, world * B_LOCAL)
        cost, x = _shard_costs(net, x0, ctx, noise, off, off + B_LOCAL)
        idx, best, row, costs = D.select(cost, x, D.argmin_nan_last)
        flag = D.any_flag(torch.tensor([rank], dtype=torch.int32))
        out[rank] = (idx, best, row.numpy(), costs.numpy(), int(flag))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_exchange_matches_single_process():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    net, x0, ctx, noise = _pipeline(world)
    cost_all, x_all = _shard_costs(net, x0, ctx, noise, 0, world * B_LOCAL)
    i = osys.argmin(cost_all.numpy())
    for r in range(world):
        idx, best, row, costs, flag = out[r]
        np.testing.assert_array_equal(costs, cost_all.numpy())  # all-gather order = global index order
        assert idx == i and best == float(cost_all[i])
        np.testing.assert_array_equal(row, x_all[i].numpy())
        assert flag == 1  # OR over ranks (rank 1 set it)
