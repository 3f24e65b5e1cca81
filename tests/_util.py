"""Shared helpers for the parity tests (oracle side + tolerance checks)."""
import os

import numpy as np
import torch

from oracle import nets, sampler, schedule

# SURVEY §8d parity bar (fp32, injected noise)
REL_TRAJ = 1e-4
ABS_ELEM = 1e-4


def make_mlp(d, H, C, seed=0):
    torch.manual_seed(seed)
    return nets.ConditionedMLPNet(state_dim=d, horizon=H, context_dim=C).eval()


def make_unet(d, C, mults=(1, 2, 4), seed=0, cfg=True):
    torch.manual_seed(seed)
    if cfg:
        return nets.ConditionedTemporalUnet(state_dim=d, context_dim=C, dim_mults=mults).eval()
    return nets.TemporalUnet(state_dim=d, dim_mults=mults, conditioning_type="default" if C else None,
                             conditioning_embed_dim=C).eval()


def assert_traj_close(got, ref, rel=REL_TRAJ, abs_elem=ABS_ELEM, what="", spread=None):
    """per trajectory ||d||_2/||ref||_2 <= rel and elementwise |d| <= abs_elem*max(|ref|, 1).
    spread: the oracle's own elementwise spread of an ill-conditioned chain (oracle_sensitivity); the elementwise
    bar is then max(abs_elem, SPREAD_X * spread), and the measured error / spread ratio is appended to the file
    $MPCD_SPREAD_LOG names (profiles/r4_spread_ratios.tsv is the GPU run's record)."""
    got = got.detach().cpu().double().numpy()
    ref = ref.detach().cpu().double().numpy()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert np.isfinite(got).all(), f"{what}: non-finite output"
    g2 = got.reshape(-1, got.shape[-2] * got.shape[-1])
    r2 = ref.reshape(g2.shape)
    tr = np.linalg.norm(g2 - r2, axis=1) / np.maximum(np.linalg.norm(r2, axis=1), 1e-30)
    el = np.abs(got - ref) / np.maximum(np.abs(ref), 1.0)
    if spread is not None:
        abs_elem = max(abs_elem, SPREAD_X * spread)
        log = os.environ.get("MPCD_SPREAD_LOG")
        if log and spread > 0:
            with open(log, "a") as f:
                f.write(f"{what}\t{el.max():.4e}\t{spread:.4e}\t{el.max() / max(spread, 1e-30):.3f}\t{tr.max():.4e}\n")
    assert tr.max() <= rel, f"{what}: worst trajectory rel err {tr.max():.3e} (> {rel})"
    assert el.max() <= abs_elem, f"{what}: worst element err {el.max():.3e} (> {abs_elem})"
    return tr.max(), el.max()


# elementwise bar of an ill-conditioned chain (unclamped DDIM, the trained 30-step Panda / LMPC chains): this multiple
# of the oracle's own spread. Another fp32-accurate implementation (split-bf16 GEMMs, its own reduction orders)
# lands a small multiple of that one-perturbation sample away: measured at most 2.89x over every such test of the GPU
# suite (profiles/r4_spread_ratios.tsv: MLP DDIM 2.89, MLP CFG-DDIM 2.36, fused U-Net CFG-DDIM 2.11, Panda 2.02,
# LMPC 1.81), so the bar is that maximum rounded up; the trajectory bar (1e-4 relative) is not relaxed.
SPREAD_X = 3


def oracle_sensitivity(run):
    """Elementwise spread of the oracle itself when every Linear/Conv/GroupNorm rounds from fp64 instead of
    fp32 (a 1-ulp-level perturbation). Unclamped DDIM is ill-conditioned (x0 = a*x - b*eps with a, b up to
    2.6e6 at N=100), so its elementwise parity bar is this spread, not 1e-4; the trajectory bar stays."""
    import torch.nn as nn
    import torch.nn.functional as F
    ref = run()
    saved = (nn.Linear.forward, nn.Conv1d.forward, nn.ConvTranspose1d.forward, nn.GroupNorm.forward)
    nn.Linear.forward = lambda self, x: F.linear(x.double(), self.weight.double(), self.bias.double()).float()
    nn.Conv1d.forward = lambda self, x: F.conv1d(x.double(), self.weight.double(), self.bias.double(), self.stride,
                                                 self.padding).float()
    nn.ConvTranspose1d.forward = lambda self, x: F.conv_transpose1d(x.double(), self.weight.double(),
                                                                    self.bias.double(), self.stride,
                                                                    self.padding).float()
    nn.GroupNorm.forward = lambda self, x: F.group_norm(x.double(), self.num_groups, self.weight.double(),
                                                        self.bias.double(), self.eps).float()
    try:
        pert = run()
    finally:
        nn.Linear.forward, nn.Conv1d.forward, nn.ConvTranspose1d.forward, nn.GroupNorm.forward = saved
    r, p = ref.double(), pert.double()
    return ref, float(((p - r).abs() / r.abs().clamp_min(1.0)).max())


def unnormalize_np(x, mn, mx):
    """fp32 LimitsNormalizer.unnormalize with the global clip rule (normalization.py:156-167)."""
    x = np.asarray(x, dtype=np.float32)
    mn = np.asarray(mn, dtype=np.float32)
    mx = np.asarray(mx, dtype=np.float32)
    if x.max() > np.float32(1 + 1e-4) or x.min() < np.float32(-1 - 1e-4):
        x = np.clip(x, np.float32(-1), np.float32(1))
    h = (x + np.float32(1)) / np.float32(2)
    return h * (mx - mn) + mn


__all__ = ["nets", "sampler", "schedule", "make_mlp", "make_unet", "assert_traj_close", "unnormalize_np", "oracle_sensitivity"]
