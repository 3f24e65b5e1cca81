"""SURVEY §8f row 1, widened: the reference's two CartPole-LMPC trained models
(trained_models/2406400_models/1000000 and 420000_models_with_noisy_data/230000: ConditionedTemporalUnet, d=1,
C=4, N=25 exponential, fixtures by tests/golden/make_lmpc_ckpts.py) through the GPU path, called as
scripts/inference/Diffusion_MPC_Inference.py:211-245 calls them - run_CFG(context, None, 0.01, n_samples,
horizon=32, return_chain=True, ddpm_cart_pole_sample_fn, n_diffusion_steps_without_noise=5) with the checkpoint's
own schedule buffers - and the torch.manual_seed(0) noise stream injected, against the oracle chain; then one
mpc_step with the reference's linear ZOH cart-pole (Diffusion_MPC_Inference.py:39-84, the cost :357-371) against
the oracle pipeline. fp32 numerics at the §8d bar (elementwise: SPREAD_X (tests/_util.py) times the oracle's own fp64-vs-fp32
spread, as for the other trained nets), fp16 operands reported (5e-2 trajectory bound)."""
import os

import numpy as np
import pytest
import torch

from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, systems
from oracle import normalizer as onorm
from oracle import sampler as osam
from oracle import schedule as osch
from oracle import systems as osys

from ._util import assert_traj_close, oracle_sensitivity

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
MODELS = ["lmpc_2406400_1000000", "lmpc_420000_noisy_230000"]


def _load(name, dtype, **kw):
    from safetensors.torch import load_file
    from oracle import nets
    sd = load_file(os.path.join(HERE, "golden", f"{name}_ema.safetensors"))
    plan = DiffusionMPC.from_state_dict(sd, NetSpec("unet", state_dim=1, horizon=32, context_dim=4, dtype=dtype), **kw)
    net = nets.ConditionedTemporalUnet(state_dim=1, context_dim=4).eval()
    net.load_state_dict({k[6:]: v for k, v in sd.items() if k.startswith("model.")}, strict=True)
    return plan, net, {k: sd[k] for k in osch.BUFFER_NAMES}


@pytest.mark.parametrize("dtype", ["f32", "f32x3", "f16"])
@pytest.mark.parametrize("name", MODELS)
@pytest.mark.parametrize("B", [1, 64])
def test_lmpc_trained_run_cfg_matches_oracle(name, dtype, B):
    plan, net, bufs = _load(name, dtype)
    torch.manual_seed(0)
    ctx = torch.rand(1, 4) * 2 - 1
    noise = torch.stack([torch.randn(B, 32, 1) for _ in range(31)])  # x_T + 25 + 5 randn_like draws
    chain = plan.run_CFG(ctx, None, 0.01, n_samples=B, horizon=32, return_chain=True, noise=noise,
                         n_diffusion_steps_without_noise=5)
    ref, spread = oracle_sensitivity(lambda: osam.ddpm_cfg(net, bufs, ctx.expand(B, 4), 0.01, B, 32, n_wo_noise=5,
                                                           noise=noise, return_chain=True))
    assert tuple(chain.shape) == (31, B, 32, 1)
    if dtype == "f16":
        got = chain[-1].cpu()
        rel = float(((got - ref[-1]).flatten(1).norm(dim=1) / ref[-1].flatten(1).norm(dim=1)).max())
        print(f"{name} f16 B={B}: trajectory rel err {rel:.3e}")
        assert torch.isfinite(got).all() and rel <= 5e-2
    else:
        tr, el = assert_traj_close(chain, ref, spread=spread, what=f"{name} {dtype} B={B}")
        print(f"{name} {dtype} B={B}: trajectory rel {tr:.2e}, element {el:.2e} (oracle spread {spread:.2e})")


@pytest.mark.parametrize("name", MODELS)
def test_lmpc_trained_mpc_step_zoh_matches_oracle(name):
    lo, hi = np.array([-10.0]), np.array([10.0])
    cmin = np.array([-2, -3, -0.5, -3], dtype=np.float32)
    cmax = np.array([2, 3, 0.5, 3], dtype=np.float32)
    plan, net, bufs = _load(name, "f32x3", action_limits=(lo, hi), context_limits=(cmin, cmax))
    B = 256
    x0 = np.array([0.3, -0.4, 0.12, 0.5])
    noise = torch.randn(31, B, 32, 1, generator=torch.Generator().manual_seed(1))
    res = plan.mpc_step(x0, systems.get("cartpole_zoh4"), B, w=0.01, noise=noise, n_wo_noise=5)
    ctx = onorm.normalize(torch.from_numpy(x0)[None], torch.from_numpy(cmin), torch.from_numpy(cmax)).float()
    chain = osam.ddpm_cfg(net, bufs, ctx.expand(B, 4), 0.01, B, 32, n_wo_noise=5, noise=noise, return_chain=True)
    u = onorm.unnormalize(chain, torch.from_numpy(lo.astype(np.float32)), torch.from_numpy(hi.astype(np.float32)))[-1]
    cost = osys.rollout_cost("cartpole_zoh4", x0, u.double().numpy())
    np.testing.assert_allclose(res.costs.cpu().numpy(), cost, rtol=1e-4)
    i = osys.argmin(cost)
    if res.best_index != i:
        assert abs(cost[res.best_index] - cost[i]) <= 1e-4 * abs(cost[i])
