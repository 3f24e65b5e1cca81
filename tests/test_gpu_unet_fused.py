"""GPU parity of the whole-network fused U-Net (csrc/unet_fused.hip: every conv of a denoise step in one launch,
activations in LDS) against the oracle and against the layer-by-layer kernels.

Reference: ConditionedTemporalUnet.forward (temporal_unet.py:287-358), ResidualTemporalBlock / Conv1dBlock /
Downsample1d / Upsample1d (layers.py:258-355), p_mean_variance_CFG + ddpm_cart_pole_sample_fn
(diffusion_model_base.py:164-209, sample_functions.py:17-44), the build-defined CFG-DDIM.
Bars: f32x3 and f16x2 (two-term fp16, the fused program's P = 2) eps 2e-5 of |eps| max, chains at the SURVEY §8d
bar (1e-4 per trajectory and elementwise); f16 (BASELINE cfg 5's fp16 operands) reported, bounded at 2e-2 eps / 5e-2
trajectory."""
import numpy as np
import pytest
import torch

from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, force_unet_path, philox_noise
from oracle import sampler as osam
from oracle import schedule as osch

from ._util import assert_traj_close, make_unet, oracle_sensitivity

pytestmark = pytest.mark.gpu

EPS_TOL = {"f32x3": 2e-5, "f16x2": 2e-5, "f16": 2e-2}


@pytest.fixture
def fused():
    force_unet_path("fused")
    yield
    force_unet_path("auto")


def _planner(net, d, H, C, N=25, kind="exponential", dtype="f32x3"):
    return DiffusionMPC(NetSpec("unet", state_dim=d, horizon=H, context_dim=C, dtype=dtype), net.state_dict(),
                        variance_schedule=kind, n_diffusion_steps=N)


def _eps_err(got, ref):
    return float((got.cpu() - ref).abs().max()) / max(float(ref.abs().max()), 1.0)


@pytest.mark.parametrize("dtype", ["f16", "f32x3", "f16x2"])
def test_fused_h128_panda_shape(dtype, fused):
    """H = 128 (the Panda net's horizon: d = 7, C = 20): fp16 operands with two rows (both CFG branches) per workgroup,
    and the fp32-accurate three-plane form with ONE row per workgroup (its activations fit one CU's LDS only one row
    at a time: unet_fused_kernel<3, 1, 128, 8> writes each branch's eps and the CFG update runs as its own launch).
    Forward against the oracle and the layered path, a CFG-DDPM chain (noise-free tail) against the oracle at the
    dtype's bar, and Philox shard invariance."""
    d, H, C, B = 7, 128, 20, 3
    net = make_unet(d, C, seed=128)
    plan = _planner(net, d, H, C, N=25, dtype=dtype)
    form = plan.unet_form()
    assert form["fused"] and form["rows_per_workgroup"] == (2 if dtype == "f16" else 1)
    assert form["planes"] == {"f16": 1, "f32x3": 3, "f16x2": 2}[dtype]
    tol = EPS_TOL[dtype]
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, H, d, generator=g)
    ctx = torch.rand(1, C, generator=g) * 2 - 1
    for t in (0, 13, 24):
        ec, eu = plan.eps(x, t, ctx)
        tt = torch.full((B,), t, dtype=torch.long)
        with torch.no_grad():
            rc = net(x, tt, ctx.expand(B, C), torch.zeros(B, 1))
            ru = net(x, tt, ctx.expand(B, C), torch.ones(B, 1))
        e1, e2 = _eps_err(ec, rc), _eps_err(eu, ru)
        assert max(e1, e2) <= tol, f"{dtype} H=128 t={t}: {e1:.2e} {e2:.2e}"
        force_unet_path("layered")
        lc, lu = plan.eps(x, t, ctx)
        force_unet_path("fused")
        assert _eps_err(ec, lc.cpu()) <= tol and _eps_err(eu, lu.cpu()) <= tol
    full = plan.sample_trajectories(ctx, 5, H, seed=3, n_wo_noise=5)
    assert torch.equal(full[2:4], plan.sample_trajectories(ctx, 2, H, seed=3, n_wo_noise=5, global_offset=2))
    if dtype != "f16":
        Bc, N = 4, 25
        noise = torch.randn(N + 5 + 1, Bc, H, d, generator=torch.Generator().manual_seed(9))
        ref = osam.ddpm_cfg(net, osch.buffers("exponential", N), ctx.expand(Bc, C), 0.01, Bc, H, n_wo_noise=5,
                            noise=noise, return_chain=True)
        got = plan.run_CFG(ctx, None, 0.01, n_samples=Bc, horizon=H, return_chain=True, noise=noise,
                           n_diffusion_steps_without_noise=5)
        assert_traj_close(got, ref, what=f"fused {dtype} H=128 chain")


@pytest.mark.parametrize("dtype", ["f32x3", "f16x2", "f16"])
@pytest.mark.parametrize("d,H,C,B", [(1, 32, 5, 24), (1, 32, 2, 37), (1, 64, 5, 6), (4, 64, 12, 5), (4, 64, 12, 131),
                                     (2, 32, 4, 16), (7, 32, 20, 9)])
def test_fused_forward_matches_oracle_and_layered(d, H, C, B, dtype, fused):
    net = make_unet(d, C, seed=d + H + C)
    plan = _planner(net, d, H, C, N=50, dtype=dtype)
    g = torch.Generator().manual_seed(H + B)
    x = torch.randn(B, H, d, generator=g)
    for shared in (True, False):
        ctx = torch.rand(1 if shared else B, C, generator=g) * 2 - 1
        for t in (0, 31, 49):
            ec, eu = plan.eps(x, t, ctx)
            tt = torch.full((B,), t, dtype=torch.long)
            with torch.no_grad():
                rc = net(x, tt, ctx.expand(B, C), torch.zeros(B, 1))
                ru = net(x, tt, ctx.expand(B, C), torch.ones(B, 1))
            e1, e2 = _eps_err(ec, rc), _eps_err(eu, ru)
            assert max(e1, e2) <= EPS_TOL[dtype], f"{dtype} d={d} H={H} B={B} t={t} shared={shared}: {e1:.2e} {e2:.2e}"
            force_unet_path("layered")
            lc, lu = plan.eps(x, t, ctx)
            force_unet_path("fused")
            assert _eps_err(ec, lc.cpu()) <= EPS_TOL[dtype] and _eps_err(eu, lu.cpu()) <= EPS_TOL[dtype]


@pytest.mark.parametrize("dtype", ["f32x3", "f16x2", "f16"])
@pytest.mark.parametrize("B,H,d,C,N,nwo,sched", [(8, 64, 1, 5, 25, 0, "exponential"), (5, 32, 1, 5, 25, 5, "exponential"),
                                                 (6, 64, 4, 12, 50, 0, "cosine"), (33, 32, 1, 2, 100, 0, "exponential")])
def test_fused_cfg_ddpm_matches_oracle(B, H, d, C, N, nwo, sched, dtype, fused):
    net = make_unet(d, C, seed=3)
    plan = _planner(net, d, H, C, N=N, kind=sched, dtype=dtype)
    g = torch.Generator().manual_seed(9)
    ctx = torch.rand(B, C, generator=g) * 2 - 1
    S = N + nwo
    noise = torch.randn(S + 1, B, H, d, generator=g)
    ref = osam.ddpm_cfg(net, osch.buffers(sched, N), ctx, 0.01, B, H, nwo, noise=noise, return_chain=True)
    am = torch.empty(B, dtype=torch.float32, device="cuda")
    got = plan.sample_trajectories(ctx, B, H, w=0.01, n_wo_noise=nwo, noise=noise, return_chain=True)
    x = plan.sample_trajectories(ctx, B, H, w=0.01, n_wo_noise=nwo, noise=noise, absmax_out=am)
    assert torch.equal(x, got[-1])
    if dtype == "f16":
        rel = float(((got[-1].cpu() - ref[-1]).flatten(1).norm(dim=1) / ref[-1].flatten(1).norm(dim=1)).max())
        print(f"fused f16 B={B} H={H} d={d} N={N}: final trajectory rel err {rel:.3e}")
        assert rel <= 5e-2
    else:
        assert_traj_close(got, ref, what=f"fused ddpm B={B} H={H}")
        assert torch.allclose(am.cpu(), ref.abs().amax(dim=(0, 2, 3)), rtol=1e-4, atol=1e-4)


def test_fused_cfg_ddim_matches_oracle(fused):
    B, H, d, C, N = 20, 32, 1, 2, 100
    net = make_unet(d, C, seed=5)
    plan = _planner(net, d, H, C, N=N)
    ctx = torch.rand(1, C, generator=torch.Generator().manual_seed(2)) * 2 - 1
    S = len(osam.ddim_grid(N, N))
    noise = torch.randn(S + 1, B, H, d, generator=torch.Generator().manual_seed(4))
    ref, spread = oracle_sensitivity(lambda: osam.ddim_cfg(net, osch.buffers("exponential", N), ctx.expand(B, C), 0.01,
                                                           B, H, noise=noise, sampling_steps=N, return_chain=True))
    got = plan.sample_trajectories(ctx, B, H, w=0.01, sample_fn="ddim_cfg", ddim_steps=N, noise=noise, return_chain=True)
    assert_traj_close(got[: ref.shape[0]], ref, spread=spread, what="fused ddim_cfg")


@pytest.mark.parametrize("dtype,H,d,C", [("f32x3", 32, 1, 2), ("f16", 64, 4, 12), ("f32x3", 64, 1, 5), ("f16x2", 32, 1, 2),
                                         ("f16x2", 64, 1, 5)])
def test_fused_philox_shards_and_layered_agree(dtype, H, d, C, fused):
    """Philox mode: any split of the batch gives the same bits (the GroupNorm order does not depend on the
    workgroup), and the layer-by-layer path agrees within twice the numerics' bar (both sit within it of the
    oracle)."""
    net = make_unet(d, C, seed=8)
    plan = _planner(net, d, H, C, N=25, dtype=dtype)
    ctx = torch.rand(1, C, generator=torch.Generator().manual_seed(3)) * 2 - 1
    B = 300
    full = plan.sample_trajectories(ctx, B, H, seed=5)
    a = plan.sample_trajectories(ctx, 101, H, seed=5, global_offset=0)
    b = plan.sample_trajectories(ctx, B - 101, H, seed=5, global_offset=101)
    assert torch.equal(full, torch.cat([a, b]))
    force_unet_path("layered")
    lay = plan.sample_trajectories(ctx, B, H, seed=5)
    force_unet_path("fused")
    rel = float(((full - lay).flatten(1).norm(dim=1) / lay.flatten(1).norm(dim=1)).max())
    # each path is within the §8d bar (1e-4) of the oracle (tests above): they agree within twice that
    assert rel <= (5e-2 if dtype == "f16" else 2e-4), rel


def test_fused_forced_on_uncovered_net_raises():
    net = make_unet(2, 3, mults=(1, 2, 4, 8), seed=1)
    plan = DiffusionMPC(NetSpec("unet", 2, 64, 3, dim_mults=(1, 2, 4, 8), dtype="f32x3"), net.state_dict(),
                        variance_schedule="cosine", n_diffusion_steps=10)
    force_unet_path("fused")
    try:
        with pytest.raises(Exception, match="fused"):
            plan.sample_trajectories(torch.zeros(1, 3), 4, 64)
    finally:
        force_unet_path("auto")
    assert torch.isfinite(plan.sample_trajectories(torch.zeros(1, 3), 4, 64)).all()


def test_f16x2_out_of_range_reruns_in_f32x3():
    """The fused U-Net's two-term fp16 program (P = 2) computes in the fp16 range. Every ResidualTemporalBlock's
    cond projection x 1e6 puts the conv inputs after it far above 65,504 (GroupNorm comes before that add): the
    P = 2 chain comes back with a NaN, the planner re-runs the call with the net's split-bf16 program (mpcd_force_f32x3)
    and returns exactly what an f32x3 plan of the same weights returns; mpcd_mpc_step does the same by itself."""
    from mpc_via_diffusion_model_amd import _native as N_
    from mpc_via_diffusion_model_amd import systems
    d, H, C, B, N = 1, 32, 5, 16, 25
    net = make_unet(d, C, seed=3)
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.Sequential) and len(m) >= 2 and isinstance(m[1], torch.nn.Linear) and \
                    isinstance(m[0], torch.nn.Mish):
                m[1].weight.mul_(1e6)
    p16 = DiffusionMPC(NetSpec("unet", d, H, C, dtype="f16x2"), net.state_dict(), n_diffusion_steps=N)
    p32 = DiffusionMPC(NetSpec("unet", d, H, C, dtype="f32x3"), net.state_dict(), n_diffusion_steps=N)
    assert p16.unet_form()["planes"] == 2 and p16.unet_form()["fused"]
    ctx = torch.rand(1, C, generator=torch.Generator().manual_seed(1)) * 2 - 1
    a = p16.sample_trajectories(ctx, B, H, seed=3)
    assert p16.last_f32x3_rerun, "the two-term fp16 program should have left the fp16 range here"
    b = p32.sample_trajectories(ctx, B, H, seed=3)
    torch.cuda.synchronize()
    assert torch.isfinite(a).all() and torch.equal(a, b)
    x0 = np.random.default_rng(2).uniform(-1, 1, C)
    r = p16.mpc_step(x0, systems.get("cartpole_nl5"), B, w=0.01, seed=5)
    r_ref = p32.mpc_step(x0, systems.get("cartpole_nl5"), B, w=0.01, seed=5)
    assert r.flags & N_.MPCD_STEP_F32X3_RERUN
    assert r.best_index == r_ref.best_index and r.best_cost == r_ref.best_cost and torch.equal(r.u_norm, r_ref.u_norm)
