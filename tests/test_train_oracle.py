"""CPU checks of the training-step oracle (oracle/train.py) the GPU trainer is compared with: the reference's
draw order, q_sample + WeightedL2, and the trainer's EMA schedule (trainer.py:302-308)."""
import torch

from oracle import schedule as osch
from oracle.train import OracleTrainer

from ._util import make_mlp


def _batch(B=16, H=8, d=2, C=3, seed=1):
    g = torch.Generator().manual_seed(seed)
    x0 = torch.rand(B, H, d, generator=g) * 2 - 1
    ctx = torch.rand(B, C, generator=g) * 2 - 1
    t = torch.randint(0, 50, (B,), generator=g)
    noise = torch.randn(B, H, d, generator=g)
    mask = torch.bernoulli(torch.zeros(B, 1) + 0.25, generator=g)
    return x0, ctx, t, noise, mask


def test_loss_is_mse_of_eps_on_q_sample():
    net = make_mlp(2, 8, 3, seed=2)
    tabs = osch.buffers("exponential", 50)
    orc = OracleTrainer(net, tabs)
    x0, ctx, t, noise, mask = _batch()
    xn = tabs["sqrt_alphas_cumprod"][t][:, None, None] * x0 + tabs["sqrt_one_minus_alphas_cumprod"][t][:, None, None] * noise
    with torch.no_grad():
        ref = ((net(xn, t, ctx, mask) - noise) ** 2).mean()
        assert torch.equal(orc.loss(x0, ctx, t, noise, mask), ref)


def test_ema_schedule():
    net = make_mlp(2, 8, 3, seed=3).train()
    orc = OracleTrainer(net, osch.buffers("exponential", 50), step_start_ema=2, update_ema_every=2, ema_decay=0.5)
    w = lambda m: m.state_dict()["final_layer.0._network.2.bias"].clone()  # noqa: E731
    b = _batch()
    orc.train_step(*b)  # step 0 < step_start_ema: reset to the model, blend -> the model (to rounding)
    assert torch.allclose(w(orc.ema), w(orc.net), atol=1e-7)
    p1 = w(orc.net)
    orc.train_step(*b)  # step 1: no EMA update
    assert torch.allclose(w(orc.ema), p1, atol=1e-7)
    orc.train_step(*b)  # step 2 >= step_start_ema: ema = 0.5 ema + 0.5 p
    assert torch.allclose(w(orc.ema), 0.5 * p1 + 0.5 * w(orc.net), atol=1e-7)
