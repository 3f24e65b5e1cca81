"""GPU parity: fp64 rollout/cost kernel vs the C oracle, unnormalise clip rule, argmin, mpc_step."""
import ctypes

import numpy as np
import pytest
import torch

from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, systems
from oracle import sampler as osam
from oracle import schedule as osch
from oracle import systems as osys

from ._util import make_mlp, make_unet, unnormalize_np

pytestmark = pytest.mark.gpu

EXACT = {"cartpole_lin5", "cartpole_zoh4", "double_int2d"}  # no transcendental: bit-exact
# sin/cos differ from glibc by <= 1 ulp (ocml vs libm); the rollouts amplify that a little over 32 steps.
RTOL = {"cartpole_nl5": 1e-9, "pendulum": 1e-9, "quadrotor12": 1e-9}


def _planner(d=1, H=32, C=5, lo=-1.0, hi=1.0):
    net = make_mlp(d, H, C)
    return DiffusionMPC(NetSpec("mlp", state_dim=d, horizon=H, context_dim=C), net.state_dict(),
                        n_diffusion_steps=25, action_limits=(np.full(d, lo), np.full(d, hi)))


def _x0(name, rng):
    n = systems.get(name).n_x
    x = rng.uniform(-1, 1, n)
    if name.startswith("cartpole") and n == 5:
        x[2] = 0.9 * np.pi + 0.1 * x[2]
        x[4] = (x[2] - np.pi) ** 2 / -np.pi + np.pi
    return x


@pytest.mark.parametrize("name", sorted(systems.REGISTRY))
@pytest.mark.parametrize("spread", [0.9, 1.3])  # 1.3: global clip rule triggers
def test_rollout_cost_matches_c_oracle(name, spread):
    sysd = systems.get(name)
    rng = np.random.default_rng(5)
    B, H = 1000, 32
    lo, hi = (-0.5, 0.3) if name == "quadrotor12" else (-3.0, 2.0)
    plan = _planner(d=sysd.n_u, H=H, C=2, lo=lo, hi=hi)
    x0 = _x0(name, rng)
    u_norm = rng.uniform(-spread, spread, (B, H, sysd.n_u)).astype(np.float32)
    u_dev = torch.from_numpy(u_norm).cuda()
    got = plan.rollout_cost(sysd, x0, u_dev).cpu().numpy()
    u = unnormalize_np(u_norm, np.full(sysd.n_u, lo), np.full(sysd.n_u, hi)).astype(np.float64)
    ref = osys.rollout_cost(name, x0, u)
    if name in EXACT:
        np.testing.assert_array_equal(got, ref)
    else:
        np.testing.assert_allclose(got, ref, rtol=RTOL[name], atol=0)


def test_calmpccost_kat5_on_gpu():
    """SURVEY §8c KAT5 (calMPCCost golden 1154598.1625456358): the C oracle reproduces the golden on u,
    and the GPU kernel equals the C oracle bit for bit on the same (unnormalised, globally clipped) input."""
    torch.manual_seed(0)
    u = torch.randn(1, 32, 1) * 5
    plan = _planner(d=1, H=32, C=2, lo=-5.0, hi=5.0)
    red = lambda th: (th - np.pi) ** 2 / -np.pi + np.pi  # noqa: E731
    x0 = np.array([0.5, 0, 0.9 * np.pi, 0, red(0.9 * np.pi)])
    u_norm = (u / 5).numpy().astype(np.float32)
    got = plan.rollout_cost(systems.cartpole_lin5(), x0, torch.from_numpy(u_norm).cuda()).cpu().numpy()
    ref = osys.rollout_cost("cartpole_lin5", x0, unnormalize_np(u_norm, [-5.0], [5.0]).astype(np.float64))
    np.testing.assert_array_equal(got, ref)
    assert osys.rollout_cost("cartpole_lin5", x0, u.double().numpy())[0] == 1154598.1625456358


def test_unnormalize_global_clip_rule():
    plan = _planner(d=2, H=16, C=2, lo=-2.0, hi=3.0)
    rng = np.random.default_rng(1)
    for spread in (0.99, 1.00005, 1.0002, 1.5):
        x = rng.uniform(-spread, spread, (37, 16, 2)).astype(np.float32)
        x[0, 0, 0] = spread
        got = plan.unnormalize_states(torch.from_numpy(x).cuda()).cpu().numpy()
        ref = unnormalize_np(x, [-2.0, -2.0], [3.0, 3.0])
        np.testing.assert_array_equal(got, ref)


def test_argmin_nan_and_ties():
    plan = _planner()
    c = torch.tensor([5.0, float("nan"), 1.0, 3.0, 1.0, float("nan")], dtype=torch.float64).cuda()
    assert plan.argmin(c) == (2, 1.0)
    assert plan.argmin(c, index_offset=100) == (102, 1.0)
    allnan = torch.full((7,), float("nan"), dtype=torch.float64).cuda()
    idx, v = plan.argmin(allnan)
    assert idx == 0 and v == float("inf")
    big = torch.rand(100003, dtype=torch.float64) + 1
    big[77777] = 0.5
    big[99999] = 0.5
    assert plan.argmin(big.cuda()) == (77777, 0.5)


@pytest.mark.parametrize("native", [False, True])
@pytest.mark.parametrize("B", [128, 100])
def test_mpc_step_matches_oracle_pipeline(native, B):
    """normalise -> CFG-DDPM sample -> unnormalise -> rollout/cost -> argmin, vs the oracle; native =
    the one-call mpcd_mpc_step (fused rollout + argmin + winner row), else the composed entry points."""
    d, H, C, N = 1, 32, 5, 25
    net = make_mlp(d, H, C, seed=9)
    lo, hi = np.array([-20.0]), np.array([20.0])
    cmin = np.array([-5, -5, 2, -5, 0], dtype=np.float32)
    cmax = np.array([5, 5, 4.5, 5, 3.2], dtype=np.float32)
    plan = DiffusionMPC(NetSpec("mlp", state_dim=d, horizon=H, context_dim=C), net.state_dict(),
                        n_diffusion_steps=N, action_limits=(lo, hi), context_limits=(cmin, cmax))
    red = lambda th: (th - np.pi) ** 2 / -np.pi + np.pi  # noqa: E731
    x0 = np.array([0.3, 0.1, 0.95 * np.pi, -0.2, red(0.95 * np.pi)])
    noise = torch.randn(N + 1, B, H, d, generator=torch.Generator().manual_seed(1))
    res = plan.mpc_step(x0, systems.cartpole_lin5(), B, w=0.01, noise=noise, native=native)
    # oracle pipeline: run_CFG(return_chain=True) -> unnormalize_states(chain) -> chain[-1]
    # (Cart_Diffusion_inference.py:450-465: the clip test sees the whole chain, x_T included)
    from oracle import normalizer as onorm
    ctx = onorm.normalize(torch.from_numpy(x0)[None], torch.from_numpy(cmin), torch.from_numpy(cmax)).float()
    chain = osam.ddpm_cfg(net, osch.buffers("exponential", N), ctx.expand(B, C), 0.01, B, H, noise=noise,
                          return_chain=True)
    u = onorm.unnormalize(chain, torch.from_numpy(lo.astype(np.float32)), torch.from_numpy(hi.astype(np.float32)))[-1]
    cost = osys.rollout_cost("cartpole_lin5", x0, u.double().numpy())
    i = osys.argmin(cost)
    gpu_cost = res.costs.cpu().numpy()
    # the cost kernel is bit-exact on the GPU's own samples (clipped, as the chain rule says)
    u_gpu = np.clip(res.u_norm.cpu().numpy(), np.float32(-1), np.float32(1))
    u_gpu = ((u_gpu + np.float32(1)) / np.float32(2)) * (hi - lo).astype(np.float32) + lo.astype(np.float32)
    np.testing.assert_array_equal(gpu_cost, osys.rollout_cost("cartpole_lin5", x0, u_gpu.astype(np.float64)))
    # and within the SURVEY §8d bar of the oracle's (sampler rounding moves these costs by ~3e-8 relative)
    np.testing.assert_allclose(gpu_cost, cost, rtol=1e-4)
    if res.best_index != i:  # only acceptable when the two costs tie within the parity bar
        assert abs(cost[res.best_index] - cost[i]) <= 1e-4 * abs(cost[i])
    np.testing.assert_allclose(res.u_best, u[res.best_index].numpy(), rtol=1e-4, atol=1e-4 * 20)
    assert res.u0.shape == (d,)


@pytest.mark.parametrize("B", [64, 1000, 4096 + 17])
@pytest.mark.parametrize("sample_fn", ["ddpm_cfg", "ddim_cfg"])
@pytest.mark.parametrize("dtype", ["f32x3", "f16x2"])
def test_native_step_equals_composed_step(B, sample_fn, dtype):
    """mpcd_mpc_step (one call, fused select) gives bit-identical samples, costs, winner and trajectory
    to the step composed from sample / clip flag / rollout / argmin / unnormalise; ragged B included
    (the last rollout workgroup is partial). DDIM leaves the clip flag live (no provable bound). f16x2 DDPM: the
    fp16 kernel computes the context row's projection inside its launch (no ctx prologue) and must match the
    composed step, which runs the prologue kernel."""
    d, H, C = 2, 32, 4
    net = make_mlp(d, H, C, seed=5)
    plan = DiffusionMPC(NetSpec("mlp", d, H, C, dtype=dtype), net.state_dict(), n_diffusion_steps=25,
                        action_limits=(np.array([-2.0, -0.5]), np.array([2.0, 0.5])))
    x0 = np.array([0.4, -0.3, 0.2, -0.1])
    sysm = systems.double_int2d()
    a = plan.mpc_step(x0, sysm, B, sample_fn=sample_fn, seed=7, native=False)
    b = plan.mpc_step(x0, sysm, B, sample_fn=sample_fn, seed=7, native=True)
    assert torch.equal(a.u_norm, b.u_norm)
    assert torch.equal(a.costs, b.costs)
    assert (a.best_index, a.best_cost) == (b.best_index, b.best_cost)
    np.testing.assert_array_equal(a.u_best, b.u_best)
    np.testing.assert_array_equal(a.u0, b.u0)


def test_native_step_ties_pick_lowest_index():
    """Every candidate gets the same injected noise -> identical trajectories and costs: the fused
    argmin must return index 0 (lowest index on ties), across several rollout workgroups."""
    d, H, C, N, B = 1, 32, 5, 25, 300
    net = make_mlp(d, H, C, seed=2)
    plan = DiffusionMPC(NetSpec("mlp", d, H, C), net.state_dict(), n_diffusion_steps=N)
    noise = torch.randn(N + 1, 1, H, d, generator=torch.Generator().manual_seed(3)).expand(N + 1, B, H, d)
    x0 = np.array([0.1, 0.0, 0.2, 0.0, 0.3])
    res = plan.mpc_step(x0, systems.cartpole_lin5(), B, noise=noise, native=True)
    c = res.costs.cpu()
    assert torch.all(c == c[0])
    assert res.best_index == 0 and res.best_cost == float(c[0])


@pytest.mark.parametrize("native", [False, True])
@pytest.mark.parametrize("clip_rule", ["chain", "final"])
def test_clip_rule_cosine_250_clamped_candidates(native, clip_rule):
    """Cosine N=250: posterior_mean_coef1[0] = 1.0000888 (fp32), so a candidate whose x0 estimate is
    clamped at step 0 ends at +-1.0000888 - inside the 1e-4 tolerance of LimitsNormalizer's test. Under
    the reference composition (run_CFG(return_chain=True), unnormalize_states(chain)) x_T ~ N(0, 1) is in
    the test, the flag is set and those candidates are clipped to +-1; under the final-samples rule they
    are not. Both rules against the oracle; the chain rule keeps every action inside its limits."""
    d, H, C, N, B = 1, 32, 5, 250, 256
    net = make_mlp(d, H, C, seed=4)
    lo, hi = np.array([-3.0]), np.array([3.0])
    plan = DiffusionMPC(NetSpec("mlp", d, H, C, dtype="f32x3"), net.state_dict(), variance_schedule="cosine",
                        n_diffusion_steps=N, action_limits=(lo, hi))
    red = lambda th: (th - np.pi) ** 2 / -np.pi + np.pi  # noqa: E731
    x0 = np.array([0.3, 0.1, 0.95 * np.pi, -0.2, red(0.95 * np.pi)])
    noise = torch.randn(N + 1, B, H, d, generator=torch.Generator().manual_seed(8))
    res = plan.mpc_step(x0, systems.cartpole_lin5(), B, w=0.01, noise=noise, native=native, clip_rule=clip_rule)
    from oracle import normalizer as onorm
    ctx = onorm.normalize(torch.from_numpy(x0)[None], -torch.ones(C), torch.ones(C)).float()
    chain = osam.ddpm_cfg(net, osch.buffers("cosine", N), ctx.expand(B, C), 0.01, B, H, noise=noise, return_chain=True)
    lo32, hi32 = torch.from_numpy(lo.astype(np.float32)), torch.from_numpy(hi.astype(np.float32))
    final = chain[-1]
    assert (final.abs() > 1).any() and final.abs().max() <= 1 + 1e-4, "the case must hold clamped candidates"
    u = onorm.unnormalize(chain if clip_rule == "chain" else final, lo32, hi32)
    u = u[-1] if clip_rule == "chain" else u
    cost = osys.rollout_cost("cartpole_lin5", x0, u.double().numpy())
    np.testing.assert_allclose(res.costs.cpu().numpy(), cost, rtol=1e-4)
    i = osys.argmin(cost)
    assert res.best_index == i or abs(cost[res.best_index] - cost[i]) <= 1e-4 * abs(cost[i])
    np.testing.assert_allclose(res.u_best, u[res.best_index].numpy(), rtol=1e-4, atol=1e-4 * 3)
    if clip_rule == "chain":
        assert np.all(res.u_best >= lo[0]) and np.all(res.u_best <= hi[0])


def test_clip_flag_nan_semantics():
    """torch's x.max() / x.min() are NaN when x holds a NaN, so LimitsNormalizer does NOT clip even if other
    values are out of range; the device flag follows (code 2) and unnormalise leaves the values unclipped."""
    plan = _planner(d=2, H=16, C=2, lo=-2.0, hi=3.0)
    x = np.full((4, 16, 2), 0.5, np.float32)
    x[1, 3, 0] = 1.7
    assert int(plan.clip_flag(torch.from_numpy(x).cuda()).item()) == 1
    x[2, 5, 1] = np.nan
    assert int(plan.clip_flag(torch.from_numpy(x).cuda()).item()) == 2
    got = plan.unnormalize_states(torch.from_numpy(x).cuda()).cpu()
    from oracle import normalizer as onorm
    ref = onorm.unnormalize(torch.from_numpy(x), torch.tensor([-2.0, -2.0]), torch.tensor([3.0, 3.0]))
    assert torch.equal(got.isnan(), ref.isnan())
    assert torch.equal(got[~got.isnan()], ref[~ref.isnan()])
    assert float(got[1, 3, 0]) == float(ref[1, 3, 0]) > 3.0  # not clipped


@pytest.mark.parametrize("kind", ["mlp_f32x3", "mlp_f32", "unet_f32x3"])
def test_chain_absmax_matches_chain(kind):
    """sample_trajectories(absmax_out=...) == max |x| over run_CFG's whole chain, per candidate."""
    d, H, C, N, B = 2, 16, 4, 25, 45
    if kind.startswith("mlp"):
        net = make_mlp(d, H, C, seed=6)
        spec = NetSpec("mlp", d, H, C, dtype=kind.split("_")[1])
    else:
        net = make_unet(d, C, seed=6)
        spec = NetSpec("unet", d, H, C, dtype="f32x3")
    plan = DiffusionMPC(spec, net.state_dict(), n_diffusion_steps=N)
    ctx = torch.rand(B if kind == "mlp_f32" else 1, C) * 2 - 1
    am = torch.empty(B, dtype=torch.float32, device="cuda")
    chain = plan.sample_trajectories(ctx, B, H, seed=3, return_chain=True, absmax_out=am)
    want = chain.abs().amax(dim=(0, 2, 3))
    assert torch.equal(am, want)


@pytest.mark.parametrize("kind", ["mlp", "unet"])
def test_nonfinite_weights_fail_loudly(kind):
    """SURVEY §5 failure detection: a NaN in the weights makes every sample NaN; mpc_step must return
    MPCD_ENONFINITE (MpcdError) instead of a silently selected garbage trajectory, and a finite run reports
    its flags (clip applied under the chain rule)."""
    from mpc_via_diffusion_model_amd import _native as N
    d, H, C = 1, 32, 5
    net = make_mlp(d, H, C, seed=1) if kind == "mlp" else make_unet(d, C, seed=1)
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    spec = NetSpec(kind, d, H, C, dtype="f32x3")
    x0 = np.array([0.3, 0.1, 0.95 * np.pi, -0.2, 0.1])
    ok = DiffusionMPC(spec, sd, n_diffusion_steps=25).mpc_step(x0, systems.cartpole_lin5(), 64, seed=3)
    assert np.isfinite(ok.best_cost) and ok.flags & N.MPCD_STEP_CLIPPED  # x_T ~ N(0,1) is in the chain
    first = next(k for k in sd if k.endswith("weight") and sd[k].dim() >= 2)
    sd[first].view(-1)[0] = float("nan")
    bad = DiffusionMPC(spec, sd, n_diffusion_steps=25)
    with pytest.raises(N.MpcdError) as ei:
        bad.mpc_step(x0, systems.cartpole_lin5(), 64, seed=3)
    assert ei.value.status == N.MPCD_ENONFINITE
    fl = ctypes.c_int32()
    N.check(bad._lib.mpcd_last_step_flags(bad._ctx, ctypes.byref(fl)), "flags")
    assert fl.value & N.MPCD_STEP_NONFINITE_WINNER and fl.value & N.MPCD_STEP_NAN_SAMPLES


@pytest.mark.parametrize("layout", ["32x8", "16x8", "16x4"])
def test_chain_absmax_every_mlp_layout(layout):
    """The per-candidate chain |x| maxima (the clip rule's input) from every MLP sampler layout, shared context
    (the split-bf16 sampler's case), ragged batch: equal to the maxima of the chain itself."""
    from mpc_via_diffusion_model_amd.planner import force_mlp_layout
    d, H, C, N, B = 2, 16, 4, 25, 45
    net = make_mlp(d, H, C, seed=7)
    plan = DiffusionMPC(NetSpec("mlp", d, H, C, dtype="f32x3"), net.state_dict(), n_diffusion_steps=N)
    ctx = torch.rand(1, C) * 2 - 1
    am = torch.empty(B, dtype=torch.float32, device="cuda")
    force_mlp_layout(layout)
    try:
        chain = plan.sample_trajectories(ctx, B, H, seed=4, return_chain=True, absmax_out=am)
    finally:
        force_mlp_layout("auto")
    assert torch.equal(am, chain.abs().amax(dim=(0, 2, 3)))
