"""Noise-prediction networks (oracle; test infrastructure only).

Restates mpd/models/diffusion_models/temporal_unet.py:
  UNET_DIM_MULTS            :14-17
  TemporalUnet              :28-187   (3-arg forward(x, t, context); conditioning None/'default')
  ConditionedTemporalUnet   :189-358  (4-arg forward with the CFG context mask :296-300)
  PointUnet                 :451-550  (MLP U-Net; the reference needs H=1 and is 3-arg)

``ConditionedMLPNet`` is BUILD-DEFINED: PointUnet's layer stack
applied to the flattened trajectory [B, H*d] with ConditionedTemporalUnet's CFG
mask and c_emb = cat(t_emb, masked ctx).float(). The reference has no CFG MLP,
so its parity is against this restatement only.

Attention / self-attention variants are out of scope (no shipped checkpoint uses them).
"""
import torch
import torch.nn as nn

from .layers import (TimeEncoder, ResidualTemporalBlock, Downsample1d, Upsample1d, Conv1dBlock,
                     TemporalBlockMLP, MLP, group_norm_n_groups)

UNET_DIM_MULTS = {0: (1, 2, 4), 1: (1, 2, 4, 8)}


def _stage_dims(first, base, mults):
    dims = [first] + [base * m for m in mults]
    return list(zip(dims[:-1], dims[1:]))


class _UnetBody(nn.Module):
    """Shared layer stack of TemporalUnet / ConditionedTemporalUnet (temporal_unet.py:69-124, 230-285)."""

    def _build(self, state_dim, base, mults, time_emb_dim, cond_dim):
        stages = _stage_dims(state_dim, base, mults)
        self.time_mlp = TimeEncoder(32, time_emb_dim)
        self.downs = nn.ModuleList([])
        self.ups = nn.ModuleList([])
        n_res = len(stages)
        for i, (ci, co) in enumerate(stages):
            last = i >= n_res - 1
            # slots 2/3 are the (disabled) self-attention and cross-attention entries
            self.downs.append(nn.ModuleList([
                ResidualTemporalBlock(ci, co, cond_dim), ResidualTemporalBlock(co, co, cond_dim),
                nn.Identity(), None, Downsample1d(co) if not last else nn.Identity()]))
        mid = stages[-1][1]
        self.mid_block1 = ResidualTemporalBlock(mid, mid, cond_dim)
        self.mid_attn = nn.Identity()
        self.mid_attention = nn.Identity()
        self.mid_block2 = ResidualTemporalBlock(mid, mid, cond_dim)
        for i, (ci, co) in enumerate(reversed(stages[1:])):
            last = i >= n_res - 1
            self.ups.append(nn.ModuleList([
                ResidualTemporalBlock(co * 2, ci, cond_dim), ResidualTemporalBlock(ci, ci, cond_dim),
                nn.Identity(), None, Upsample1d(ci) if not last else nn.Identity()]))
        self.final_conv = nn.Sequential(
            Conv1dBlock(base, base, kernel_size=5, n_groups=group_norm_n_groups(base)),
            nn.Conv1d(base, state_dim, 1))

    def _trunk(self, x, c_emb):
        # x: [B, H, d] -> [B, d, H]; forward :317-356
        x = x.transpose(1, 2)
        skips = []
        for rtb1, rtb2, _sa, _ca, down in self.downs:
            x = rtb2(rtb1(x, c_emb), c_emb)
            skips.append(x)
            x = down(x)
        x = self.mid_block2(self.mid_block1(x, c_emb), c_emb)
        for rtb1, rtb2, _sa, _ca, up in self.ups:
            x = torch.cat((x, skips.pop()), dim=1)
            x = up(rtb2(rtb1(x, c_emb), c_emb))
        x = self.final_conv(x)
        return x.transpose(1, 2)


class ConditionedTemporalUnet(_UnetBody):
    def __init__(self, state_dim, context_dim, unet_input_dim=32, dim_mults=(1, 2, 4), time_emb_dim=32,
                 **_ignored):
        super().__init__()
        self.state_dim = state_dim
        self.context_dim = context_dim
        self._build(state_dim, unet_input_dim, dim_mults, time_emb_dim, time_emb_dim + context_dim)

    def forward(self, x, t, context, context_mask):
        keep = 1 * (1 - context_mask.repeat(1, context.size(1)))
        ctx = torch.mul(context, keep)
        c_emb = torch.cat((self.time_mlp(t), ctx), dim=-1).float()
        return self._trunk(x, c_emb)


class TemporalUnet(_UnetBody):
    """conditioning_type None (c_emb = t_emb) or 'default' (c_emb = cat(t_emb, context))."""

    def __init__(self, state_dim, unet_input_dim=32, dim_mults=(1, 2, 4, 8), time_emb_dim=32,
                 conditioning_type=None, conditioning_embed_dim=4, **_ignored):
        super().__init__()
        self.state_dim = state_dim
        self.conditioning_type = conditioning_type if conditioning_type not in ("None",) else None
        cond_dim = time_emb_dim + (conditioning_embed_dim if self.conditioning_type == "default" else 0)
        self.context_dim = conditioning_embed_dim if self.conditioning_type == "default" else 0
        self._build(state_dim, unet_input_dim, dim_mults, time_emb_dim, cond_dim)

    def forward(self, x, t, context=None):
        c_emb = self.time_mlp(t)
        if self.conditioning_type == "default":
            c_emb = torch.cat((c_emb, context), dim=-1)
        return self._trunk(x, c_emb)


class ConditionedMLPNet(nn.Module):
    """Build-defined CFG MLP noise-net: PointUnet stack (temporal_unet.py:489-518) on [B, H*d]."""

    def __init__(self, state_dim, horizon, context_dim, dim=32, dim_mults=(1, 2, 4), time_emb_dim=32,
                 **_ignored):
        super().__init__()
        self.state_dim = state_dim
        self.horizon = horizon
        self.context_dim = context_dim
        flat = horizon * state_dim
        cond_dim = time_emb_dim + context_dim
        stages = _stage_dims(flat, dim, dim_mults)
        self.time_mlp = TimeEncoder(32, time_emb_dim)
        self.downs = nn.ModuleList([nn.ModuleList([TemporalBlockMLP(ci, co, cond_dim)]) for ci, co in stages])
        self.ups = nn.ModuleList([])
        mid = stages[-1][1]
        self.mid_block1 = TemporalBlockMLP(mid, mid, cond_dim)
        for ci, co in reversed(stages[1:]):
            self.ups.append(nn.ModuleList([TemporalBlockMLP(co * 2, ci, cond_dim)]))
        self.final_layer = nn.Sequential(MLP(dim, flat, hidden_dim=dim, n_layers=0, act="identity"))

    def forward(self, x, t, context, context_mask):
        b, h, d = x.shape
        keep = 1 * (1 - context_mask.repeat(1, context.size(1)))
        ctx = torch.mul(context, keep)
        c_emb = torch.cat((self.time_mlp(t), ctx), dim=-1).float()
        y = x.reshape(b, h * d)
        skips = []
        for (blk,) in self.downs:
            y = blk(y, c_emb)
            skips.append(y)
        y = self.mid_block1(y, c_emb)
        for (blk,) in self.ups:
            y = blk(torch.cat((y, skips.pop()), dim=1), c_emb)
        return self.final_layer(y).reshape(b, h, d)


def param_count(module):
    return sum(p.numel() for p in module.parameters())
