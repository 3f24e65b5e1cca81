"""Noise-net building blocks (oracle; test infrastructure only).

Restates mpd/models/layers/layers.py. Module attribute names and Sequential
indices are kept so that ``state_dict()`` keys equal the reference's (the
trained checkpoints load straight in, weights-only):
  MLP               layers.py:12-35   (Linear, act, [Linear, BN, act]*n, Linear)
  TimeEncoder       layers.py:229-240 (SinusoidalPosEmb -> Linear(d,4d) -> Mish -> Linear(4d,out))
  SinusoidalPosEmb  layers.py:243-255
  Downsample1d      layers.py:258-264 (Conv1d k3 s2 p1)
  Upsample1d        layers.py:267-273 (ConvTranspose1d k4 s2 p1)
  Conv1dBlock       layers.py:276-293 (Conv1d -> GroupNorm -> Mish; index 1/3 are reshapes)
  ResidualTemporalBlock layers.py:323-355
  TemporalBlockMLP  layers.py:358-385
  group_norm_n_groups layers.py:389-395
"""
import math

import torch
import torch.nn as nn


def group_norm_n_groups(channels, target=8):
    if channels < target:
        return 1
    for g in range(target, target + 10):
        if channels % g == 0:
            return g
    return 1


class _AddUnitAxis(nn.Module):
    """[B, C, L] -> [B, C, 1, L] (the reference's einops Rearrange, no parameters)."""

    def forward(self, x):
        return x.unsqueeze(2)


class _DropUnitAxis(nn.Module):
    def forward(self, x):
        return x.squeeze(2)


class _ColumnAxis(nn.Module):
    """[B, C] -> [B, C, 1]."""

    def forward(self, x):
        return x.unsqueeze(-1)


class MLP(nn.Module):
    _ACTS = {"mish": nn.Mish, "identity": nn.Identity, "relu": nn.ReLU, "tanh": nn.Tanh}

    def __init__(self, in_dim, out_dim, hidden_dim=16, n_layers=1, act="relu", batch_norm=True):
        super().__init__()
        act_cls = self._ACTS[act]
        seq = [nn.Linear(in_dim, hidden_dim), act_cls()]
        for _ in range(n_layers):
            seq += [nn.Linear(hidden_dim, hidden_dim),
                    nn.BatchNorm1d(hidden_dim) if batch_norm else nn.Identity(), act_cls()]
        seq.append(nn.Linear(hidden_dim, out_dim))
        self._network = nn.Sequential(*seq)

    def forward(self, x):
        return self._network(x)


class SinusoidalPosEmb(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, t):
        half = self.dim // 2
        step = math.log(10000) / (half - 1)
        freqs = torch.exp(torch.arange(half, device=t.device) * -step)
        arg = t[:, None] * freqs[None, :]
        return torch.cat((arg.sin(), arg.cos()), dim=-1)


class TimeEncoder(nn.Module):
    def __init__(self, dim, dim_out):
        super().__init__()
        self.encoder = nn.Sequential(SinusoidalPosEmb(dim), nn.Linear(dim, dim * 4), nn.Mish(),
                                     nn.Linear(dim * 4, dim_out))

    def forward(self, t):
        return self.encoder(t)


class Downsample1d(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.conv = nn.Conv1d(dim, dim, kernel_size=3, stride=2, padding=1)

    def forward(self, x):
        return self.conv(x)


class Upsample1d(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.conv = nn.ConvTranspose1d(dim, dim, kernel_size=4, stride=2, padding=1)

    def forward(self, x):
        return self.conv(x)


class Conv1dBlock(nn.Module):
    def __init__(self, cin, cout, kernel_size, n_groups=8):
        super().__init__()
        self.block = nn.Sequential(
            nn.Conv1d(cin, cout, kernel_size, stride=1, padding=kernel_size // 2),
            _AddUnitAxis(), nn.GroupNorm(n_groups, cout), _DropUnitAxis(), nn.Mish())

    def forward(self, x):
        return self.block(x)


class ResidualTemporalBlock(nn.Module):
    def __init__(self, cin, cout, cond_dim, kernel_size=5):
        super().__init__()
        g = group_norm_n_groups(cout)
        self.blocks = nn.ModuleList([Conv1dBlock(cin, cout, kernel_size, n_groups=g),
                                     Conv1dBlock(cout, cout, kernel_size, n_groups=g)])
        self.cond_mlp = nn.Sequential(nn.Mish(), nn.Linear(cond_dim, cout), _ColumnAxis())
        self.residual_conv = nn.Conv1d(cin, cout, 1) if cin != cout else nn.Identity()

    def forward(self, x, c):
        h = self.blocks[0](x) + self.cond_mlp(c)
        h = self.blocks[1](h)
        return h + self.residual_conv(x)


class TemporalBlockMLP(nn.Module):
    def __init__(self, cin, cout, cond_dim):
        super().__init__()
        self.blocks = nn.ModuleList([MLP(cin, cout, hidden_dim=cout, n_layers=0, act="mish")])
        self.cond_mlp = nn.Sequential(nn.Mish(), nn.Linear(cond_dim, cout))
        self.last_act = nn.Mish()

    def forward(self, x, c):
        return self.last_act(self.blocks[0](x) + self.cond_mlp(c))
