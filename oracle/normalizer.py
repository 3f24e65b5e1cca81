"""LimitsNormalizer semantics (oracle; test infrastructure only).

Restates mpd/datasets/normalization.py:144-167 with the dtypes the control loop uses
(scripts/inference/Cart_Diffusion_inference.py:405-410, mpd/datasets/cart_pole_u.py:185-201):
the state x0 is float64 and the dataset min/max are float32, so ``normalize`` runs in fp64
(and the net casts c_emb to fp32, temporal_unet.py:314); ``unnormalize`` runs on the fp32
sample and clips ONLY when the global max/min of the whole tensor leaves [-1-eps, 1+eps].
"""
import torch


def normalize(x0_f64, mins_f32, maxs_f32):
    x = (x0_f64 - mins_f32) / (maxs_f32 - mins_f32)
    return 2 * x - 1


def unnormalize(x_f32, mins_f32, maxs_f32, eps=1e-4):
    if x_f32.max() > 1 + eps or x_f32.min() < -1 - eps:
        x_f32 = torch.clip(x_f32, -1, 1)
    x = (x_f32 + 1) / 2.0
    return x * (maxs_f32 - mins_f32) + mins_f32
