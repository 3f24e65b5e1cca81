"""GPU parity of the two-term fp16 MLP sampler (MPCD_F16X2, csrc/mlp_h2.hip) beyond the shared MLP suite
(tests/test_gpu_mlp.py runs every oracle case with dtype "f16x2" too): the kernel that runs is the h2 kernel where
it applies and the f32x3 / f32 kernels where it does not; its two workgroup forms (32 and 16 rows) give the same
bits; full-size agreement with the exact-fp32 kernel; the per-layer weight scales keep tiny and large weights
to the bar; large and tiny activations meet the bar; a net whose activations leave the fp16 range is re-run with the
net's split-bf16 kernels (planner and mpcd_mpc_step), never returned as a NaN or a silently wrong value. f16x2 is
22-bit operands in the fp16 range, NOT fp32 arithmetic (include/mpcd.h). Reference net: temporal_unet.py:451-550 / layers.py:358-385 (SURVEY A11,
build-defined CFG MLP)."""
import numpy as np
import pytest
import torch

from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec
from oracle import sampler as osam
from oracle import schedule as osch

from ._util import assert_traj_close, make_mlp

pytestmark = pytest.mark.gpu


def _plan(net, d, H, C, N=100, dtype="f16x2"):
    return DiffusionMPC(NetSpec("mlp", state_dim=d, horizon=H, context_dim=C, dtype=dtype), net.state_dict(),
                        variance_schedule="exponential", n_diffusion_steps=N)


def _ctx(C, seed=3):
    return torch.rand(1, C, generator=torch.Generator().manual_seed(seed)) * 2 - 1


def test_kernel_choice():
    H, d, C = 32, 2, 4
    plan = _plan(make_mlp(d, H, C), d, H, C)
    assert plan.mlp_form(4096) == {"kernel": "h2", "layout": None, "rows_per_workgroup": 32}
    assert plan.mlp_form(512)["rows_per_workgroup"] == 16 and plan.mlp_form(512)["kernel"] == "h2"
    assert plan.mlp_form(4096, "ddim_cfg")["kernel"] == "x3"  # unclamped DDIM: the bf16x3 kernels
    big = _plan(make_mlp(2, 64, C), 2, 64, C)                 # H*d = 128
    assert big.mlp_form(64)["kernel"] == "x3"


@pytest.mark.parametrize("B,H", [(4096, 32), (333, 32), (64, 16)])
def test_row_forms_bit_identical(B, H):
    """32-row and 16-row workgroups (forced through the bf16x3 layout switch, which the h2 kernel follows) compute the
    same sums in the same order: identical chains, Philox noise, full cfg2 size and a ragged batch."""
    from mpc_via_diffusion_model_amd.planner import force_mlp_layout
    d, C = 2, 4
    plan = _plan(make_mlp(d, H, C, seed=5), d, H, C)
    ctx = _ctx(C)
    outs = {}
    try:
        for lay in ("rw32", "rw16"):
            force_mlp_layout(lay)
            assert plan.mlp_form(B)["rows_per_workgroup"] == (32 if lay == "rw32" else 16)
            outs[lay] = plan.run_CFG(ctx, None, 0.01, n_samples=B, horizon=H, return_chain=True, seed=3)
            torch.cuda.synchronize()
    finally:
        force_mlp_layout("auto")
    assert torch.isfinite(outs["rw32"]).all()
    assert torch.equal(outs["rw32"], outs["rw16"]), float((outs["rw32"] - outs["rw16"]).abs().max())


def test_full_size_against_exact_f32():
    """cfg2 size, Philox noise: the two-term fp16 kernel against the exact-fp32 MFMA kernel (same seed)."""
    B, H, d, C, N = 4096, 32, 2, 4, 100
    net = make_mlp(d, H, C, seed=21)
    ctx = _ctx(C)
    a = _plan(net, d, H, C, N, dtype="f32").sample_trajectories(ctx, B, H, seed=9)
    b = _plan(net, d, H, C, N).sample_trajectories(ctx, B, H, seed=9)
    torch.cuda.synchronize()
    assert torch.isfinite(b).all()
    rel = (a - b).flatten(1).norm(dim=1) / a.flatten(1).norm(dim=1).clamp_min(1e-12)
    el = (a - b).abs().max()
    print(f"f16x2 vs exact f32 at B=4096: worst trajectory rel {float(rel.max()):.3e}, worst element {float(el):.3e}")
    assert float(rel.max()) < 1e-4 and float(el) < 1e-4


def _oracle_and_gpu(net, d, H, C, N, B, seed=11):
    plan = _plan(net, d, H, C, N)
    ctx = _ctx(C)
    noise = torch.randn(N + 1, B, H, d, generator=torch.Generator().manual_seed(seed))
    ref = osam.ddpm_cfg(net, osch.buffers("exponential", N), ctx.expand(B, C), 0.01, B, H, noise=noise,
                        return_chain=True)
    got = plan.run_CFG(ctx, None, 0.01, n_samples=B, horizon=H, return_chain=True, noise=noise)
    torch.cuda.synchronize()
    return plan, ref, got


def _scaled_mlp(d, H, C, seed, weight=1.0, first=None, bias=None):
    """make_mlp with every Linear weight x `weight` but the final layer's (first: the input layer's factor instead;
    bias: every Linear bias x `bias`)"""
    net = make_mlp(d, H, C, seed=seed)
    lins = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    with torch.no_grad():
        for m in lins:
            if m.weight.shape[0] == H * d:
                continue  # the final Linear (flat output)
            f = first if (first is not None and m.weight.shape[1] == H * d) else (weight if first is None else 1.0)
            m.weight.mul_(f)
            if bias is not None:
                m.bias.mul_(bias)
    return net


@pytest.mark.parametrize("scale", [1e-3, 30.0])
def test_weight_scales(scale):
    """Per-layer power-of-two weight scaling: a net with every Linear weight x 1e-3 (lo terms would be fp16
    subnormals unscaled) or x 30 (hi terms near the fp16 range unscaled) meets the oracle at the bar - a hard
    assertion: an f16x2 call that leaves the fp16 range is re-run with the net's split-bf16 kernels (planner)."""
    B, H, d, C, N = 128, 32, 2, 4, 100
    plan, ref, got = _oracle_and_gpu(_scaled_mlp(d, H, C, 7, weight=scale), d, H, C, N, B)
    assert torch.isfinite(ref).all(), "the oracle itself must stay finite at this scale"
    assert torch.isfinite(got).all()
    tr, el = assert_traj_close(got, ref, what=f"f16x2, weights x {scale}")
    print(f"weights x {scale}: f32x3 re-run {plan.last_f32x3_rerun}, worst trajectory {tr:.3e}, element {el:.3e}")


def test_large_activations():
    """Input-layer weights x 100: first-layer activations two orders of magnitude up (|v| into the thousands)."""
    B, H, d, C, N = 128, 32, 2, 4, 100
    plan, ref, got = _oracle_and_gpu(_scaled_mlp(d, H, C, 8, first=100.0), d, H, C, N, B)
    assert torch.isfinite(ref).all() and torch.isfinite(got).all()
    tr, el = assert_traj_close(got, ref, what="f16x2, input layer x 100")
    print(f"input layer x 100: f32x3 re-run {plan.last_f32x3_rerun}, worst trajectory {tr:.3e}, element {el:.3e}")


def test_small_activations():
    """Biases zeroed and every hidden weight x 1e-2: activations shrink ~100x per layer, deep into the fp16 subnormal
    range (absolute precision 2^-25 there); their contribution to eps shrinks with them."""
    B, H, d, C, N = 128, 32, 2, 4, 100
    plan, ref, got = _oracle_and_gpu(_scaled_mlp(d, H, C, 9, weight=1e-2, bias=0.0), d, H, C, N, B)
    assert torch.isfinite(ref).all() and torch.isfinite(got).all()
    tr, el = assert_traj_close(got, ref, what="f16x2, biases 0, weights x 1e-2")
    print(f"small activations: f32x3 re-run {plan.last_f32x3_rerun}, worst trajectory {tr:.3e}, element {el:.3e}")


def test_out_of_range_reruns_in_f32x3():
    """A net whose activations certainly leave the fp16 range (hidden weights x 1e4, final layer x 1e-8 so the oracle's
    eps stays moderate): the f16x2 chain would hold NaN; the planner re-runs the call with the split-bf16 kernels
    (bit-identical to an f32x3 plan of the same weights), and mpcd_mpc_step does the same by itself
    (MPCD_STEP_F32X3_RERUN)."""
    from mpc_via_diffusion_model_amd import _native as N_
    from mpc_via_diffusion_model_amd import systems
    B, H, d, C, N = 64, 32, 2, 4, 50
    net = _scaled_mlp(d, H, C, 10, first=1e4)
    with torch.no_grad():
        lins = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
        lins[-1].weight.mul_(1e-8)
    plan = _plan(net, d, H, C, N)
    ref_plan = _plan(net, d, H, C, N, dtype="f32x3")
    ctx = _ctx(C)
    got = plan.sample_trajectories(ctx, B, H, seed=4)
    assert plan.last_f32x3_rerun, "the f16x2 kernel should have left the fp16 range here"
    want = ref_plan.sample_trajectories(ctx, B, H, seed=4)
    torch.cuda.synchronize()
    assert torch.isfinite(got).all() and torch.equal(got, want)
    x0 = np.random.default_rng(1).uniform(-1, 1, C)
    r = plan.mpc_step(x0, systems.get("double_int2d"), B, w=0.01, seed=6)
    r_ref = ref_plan.mpc_step(x0, systems.get("double_int2d"), B, w=0.01, seed=6)
    assert r.flags & N_.MPCD_STEP_F32X3_RERUN and not (r_ref.flags & N_.MPCD_STEP_F32X3_RERUN)
    assert r.best_index == r_ref.best_index and r.best_cost == r_ref.best_cost
    assert torch.equal(r.u_norm, r_ref.u_norm)
