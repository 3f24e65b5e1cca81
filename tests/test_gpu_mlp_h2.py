"""GPU parity of the two-term fp16 MLP sampler (MPCD_F16X2, csrc/mlp_h2.hip) beyond the shared MLP suite
(tests/test_gpu_mlp.py runs every oracle case with dtype "f16x2" too): the kernel that runs is the h2 kernel where
it applies and the f32x3 / f32 kernels where it does not; its two workgroup forms (32 and 16 rows) give the same
bits; full-size agreement with the exact-fp32 kernel; the per-layer weight scales keep tiny and large weights
exact to the bar; a net whose activations leave the fp16 range gives a non-finite sample, which the chain |x|
maximum reports (no silent wrong value). Reference net: temporal_unet.py:451-550 / layers.py:358-385 (SURVEY A11,
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


@pytest.mark.parametrize("scale", [1e-3, 30.0])
def test_weight_scales(scale):
    """Per-layer power-of-two weight scaling: a net with every Linear weight x 1e-3 (lo terms would be fp16
    subnormals unscaled) or x 30 (hi terms near the fp16 range unscaled) still meets the oracle at the bar."""
    B, H, d, C, N = 128, 32, 2, 4, 100
    net = make_mlp(d, H, C, seed=7)
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.Linear):
                m.weight.mul_(scale if m.weight.shape[0] != H * d else 1.0)
    plan = _plan(net, d, H, C, N)
    ctx = _ctx(C)
    noise = torch.randn(N + 1, B, H, d, generator=torch.Generator().manual_seed(11))
    ref = osam.ddpm_cfg(net, osch.buffers("exponential", N), ctx.expand(B, C), 0.01, B, H, noise=noise,
                        return_chain=True)
    got = plan.run_CFG(ctx, None, 0.01, n_samples=B, horizon=H, return_chain=True, noise=noise)
    if not torch.isfinite(ref).all():
        pytest.skip("the oracle itself overflows at this scale")
    if not torch.isfinite(got).all():
        # activations beyond the fp16 range: reported as non-finite, never silently wrong
        amax = torch.empty(B, dtype=torch.float32, device=plan.device)
        plan.sample_trajectories(ctx, B, H, noise=noise, absmax_out=amax)
        assert torch.isnan(amax).any() or torch.isinf(amax).any()
        return
    assert_traj_close(got, ref, what=f"f16x2, weights x {scale}")
