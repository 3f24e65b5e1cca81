"""GPU parity of the EXACT path the bench times, at full size, against the oracle.

bench.py's step is `plan.mpc_step(x0, double_int2d, B, w=0.01, seed=...)` with in-kernel Philox noise, the
default (auto) MLP workgroup layout, the native one-call step (mpcd_mpc_step: sampler, chain-wide clip flag,
fp64 rollout/cost fused with the argmin, winner row). Here that same call runs at BASELINE cfg 2 (B=4096,
H=32, N=100) and cfg 1 (B=64, H=16, N=50) for both MLP numerics: f32x3, the bench default (the resident-weight
split-bf16 `mlp_rw_kernel<64, DDPM_CFG, ctx, 32>` at cfg 2, its 16-row form `mlp_rw_kernel<32, DDPM_CFG, ctx, 16>`
at cfg 1) and f16x2 (`mlp_h2_kernel<64, DDPM_CFG, ctx, 32>` / `<32, DDPM_CFG, ctx, 16>`, --dtype f16x2); every
candidate's Philox draws are replayed (mpcd_philox_noise) through the oracle
sampler (diffusion_model_base.py:181-209, sample_functions.py:17-44), the oracle LimitsNormalizer's
chain-wide clip rule (normalization.py:156-167) and the C cost oracle, then argmin
(scripts/inference/inference_(mpd).py:335-338). Bars: samples per trajectory 1e-4 and
elementwise 1e-4, costs rtol 1e-4, argmin identical or tied within 1e-4.
"""
import numpy as np
import pytest
import torch

from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, philox_noise, systems
from oracle import normalizer as onorm
from oracle import sampler as osam
from oracle import schedule as osch
from oracle import systems as osys

from ._util import assert_traj_close, make_mlp

pytestmark = pytest.mark.gpu

# (B, H, d, C, N) of BASELINE configs[0] / configs[1] (bench.py WORKLOADS)
CASES = {"cfg1": (64, 16, 2, 4, 50), "cfg2": (4096, 32, 2, 4, 100)}


@pytest.mark.parametrize("dtype", ["f32x3", "f16x2"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_timed_mpc_step_matches_oracle_full_batch(name, dtype):
    """Both MLP numerics: the fp32-accurate split-bf16 kernels (f32x3, the bench default) and the two-term fp16 kernel
    (f16x2: 22-bit operands, fp16 range; csrc/mlp_h2.hip: mlp_h2_kernel<64, DDPM_CFG, ctx, 32> at cfg2,
    <32, DDPM_CFG, ctx, 16> at cfg1), each against the same oracle bars."""
    B, H, d, C, N = CASES[name]
    torch.set_num_threads(min(16, torch.get_num_threads()))
    net = make_mlp(d, H, C, seed=0)
    spec = NetSpec("mlp", state_dim=d, horizon=H, context_dim=C, dtype=dtype)
    plan = DiffusionMPC(spec, net.state_dict(), variance_schedule="exponential", n_diffusion_steps=N)
    assert plan.mlp_form(B)["kernel"] == ("h2" if dtype == "f16x2" else "x3")
    system = systems.get("double_int2d")
    x0 = np.random.default_rng(1).uniform(-1, 1, C)
    seed = 2
    res = plan.mpc_step(x0, system, B, w=0.01, seed=seed)  # bench.py's call, native step, Philox noise
    torch.cuda.synchronize()

    noise = philox_noise(B, N + 1, H * d, seed=seed, global_offset=0).view(N + 1, B, H, d).cpu()
    one = torch.ones(C, dtype=torch.float32)
    ctx = onorm.normalize(torch.from_numpy(x0)[None], -one, one).float()
    chain = osam.ddpm_cfg(net, osch.buffers("exponential", N), ctx.expand(B, C), 0.01, B, H, noise=noise,
                          return_chain=True)
    tr, el = assert_traj_close(res.u_norm, chain[-1], what=f"{name} timed path, full batch")
    u_all = onorm.unnormalize(chain, -torch.ones(d), torch.ones(d))  # clip test over the whole chain
    u = u_all[-1]
    cost = osys.rollout_cost("double_int2d", x0, u.double().numpy())
    got = res.costs.cpu().numpy()
    np.testing.assert_allclose(got, cost, rtol=1e-4)
    i = osys.argmin(cost)
    if res.best_index != i:
        assert abs(cost[res.best_index] - cost[i]) <= 1e-4 * abs(cost[i]), (res.best_index, i)
    assert abs(res.best_cost - cost[i]) <= 1e-4 * abs(cost[i])
    # the applied trajectory is the winner's unnormalised row
    ref_row = u[res.best_index].numpy()
    np.testing.assert_allclose(res.u_best, ref_row, rtol=0, atol=1e-4)
    print(f"{name} {dtype}: B={B} worst trajectory rel {tr:.3e}, worst element {el:.3e}, "
          f"max cost rel {float(np.max(np.abs(got - cost) / np.abs(cost))):.3e}, argmin {res.best_index} (oracle {i})")
