"""Oracle training step (TEST INFRASTRUCTURE ONLY): the reference's optimisation step restated in torch on
the CPU, fp32, over the oracle's CFG MLP noise-net.

  loss = WeightedL2(net(q_sample(x0, t, noise), t, context, context_mask), noise)
        -> mean((eps - noise)^2)                     helpers.py:71-99 (weights None), predict_epsilon
  q_sample = sqrt(abar_t) x0 + sqrt(1 - abar_t) noise  diffusion_model_base.py:421-431
  backward, torch.optim.Adam(lr)                        trainer.py:152, :284-300
  EMA every update_ema_every steps; before step_start_ema the EMA model is reset to the model first
                                                        trainer.py:70-88, :302-308
The random draws (t, noise, context_mask) are inputs, drawn by the caller in p_losses' order
(diffusion_model_base.py:434-472). Parity unpinned against the reference itself (its trainer cannot run
here); the formulas are restated from the cited lines and checked against torch autograd."""
import copy

import torch


class OracleTrainer:
    def __init__(self, net, tables, lr=3e-3, betas=(0.9, 0.999), eps=1e-8, ema_decay=0.995, step_start_ema=1000,
                 update_ema_every=10):
        self.net = net
        self.ema = copy.deepcopy(net)
        self.tables = tables
        self.opt = torch.optim.Adam(lr=lr, params=net.parameters(), betas=betas, eps=eps)
        self.beta = ema_decay
        self.step_start_ema = step_start_ema
        self.update_ema_every = update_ema_every
        self.steps = 0

    def loss(self, x0, context, t, noise, context_mask):
        sac = self.tables["sqrt_alphas_cumprod"][t].reshape(-1, 1, 1)
        s1m = self.tables["sqrt_one_minus_alphas_cumprod"][t].reshape(-1, 1, 1)
        x_noisy = sac * x0 + s1m * noise
        eps = self.net(x_noisy, t, context, context_mask.reshape(-1, 1))
        return torch.nn.functional.mse_loss(eps, noise, reduction="none").mean()

    def train_step(self, x0, context, t, noise, context_mask):
        loss = self.loss(x0, context, t, noise, context_mask)
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        if self.steps % self.update_ema_every == 0:
            if self.steps < self.step_start_ema:
                self.ema.load_state_dict(self.net.state_dict())
            with torch.no_grad():
                for pe, p in zip(self.ema.parameters(), self.net.parameters()):
                    pe.data = pe.data * self.beta + (1 - self.beta) * p.data
        self.steps += 1
        return float(loss)
