"""Native training step for the CFG MLP noise-net and ConditionedTemporalUnet behind the reference's interface:
GaussianDiffusionModel.loss(x, context) -> p_losses (mpd/models/diffusion_models/diffusion_model_base.py:
434-472) with CFG context dropout (drop_prob, :57, :449), the WeightedL2 loss (helpers.py:71-99), and the
trainer's optimisation step (mpd/trainer/trainer.py:152 Adam, :284-308 backward / step / EMA).

Everything runs in libmpcd.so (csrc/train.hip) on the device; this module only draws p_losses' random
inputs in the reference's order (randint t, randn_like noise, rand + bernoulli context mask) with torch's
RNG, so a seeded run consumes the same stream the reference does."""
import ctypes

import torch

from . import _native as N
from . import schedule as S

WHICH = {"params": 0, "ema": 1, "grads": 2, "exp_avg": 3, "exp_avg_sq": 4}


class DiffusionTrainer:
    def __init__(self, spec, params, variance_schedule="exponential", n_diffusion_steps=100, tables=None, lr=3e-3,
                 betas=(0.9, 0.999), eps=1e-8, ema_decay=0.995, step_start_ema=1000, update_ema_every=10,
                 drop_prob=0.25, device=None):
        """spec: NetSpec(kind="mlp" or "unet" with cfg=True, ...); params: state_dict of the net (no "model." prefix). Defaults are the
        reference's (NN_cart_pole_train.py:143,168-170; diffusion_model_base.py:57; torch Adam)."""
        if spec.kind not in ("mlp", "unet") or (spec.kind == "unet" and not spec.cfg):
            raise ValueError("the native training step covers the CFG MLP noise-net and ConditionedTemporalUnet")
        self.spec = spec
        self.drop_prob = float(drop_prob)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.tables = tables if tables is not None else S.tables(variance_schedule, n_diffusion_steps)
        self.n_steps = int(self.tables["betas"].numel())
        self._lib = N.lib()
        self._desc = spec.desc()
        self.param_spec = N.param_spec(self._desc)
        blob = torch.cat([params[n].detach().to("cpu", torch.float32).reshape(-1) for n, _ in self.param_spec])
        self.n_params = blob.numel()
        cfg = N.TrainCfg(lr, betas[0], betas[1], eps, ema_decay, step_start_ema, update_ema_every)
        sac = self.tables["sqrt_alphas_cumprod"].to(torch.float32).contiguous()
        s1m = self.tables["sqrt_one_minus_alphas_cumprod"].to(torch.float32).contiguous()
        self._tr = ctypes.c_void_p()
        # the trainer's buffers live on the device current at mpcd_trainer_create (every later mpcd_trainer_*
        # call switches back to it)
        with torch.cuda.device(self.device):
            N.check(self._lib.mpcd_trainer_create(ctypes.byref(self._desc), ctypes.c_void_p(blob.data_ptr()), self.n_params,
                                                  ctypes.byref(cfg), ctypes.c_void_p(sac.data_ptr()),
                                                  ctypes.c_void_p(s1m.data_ptr()), self.n_steps, ctypes.byref(self._tr)),
                    "mpcd_trainer_create")

    def data_parallel(self, group=None, loopback=None):
        """Average gradients over ranks before each Adam step (DistributedDataParallel's rule) through an RCCL
        communicator of this trainer: rank 0's unique id is shipped over the torch.distributed group (one
        process per GPU). loopback=(nranks, rank, key): a virtual rank of an in-process group on one GPU
        instead (each trainer stepped from its own host thread)."""
        if loopback is not None:
            n, r, key = (int(v) for v in loopback)
            N.check(self._lib.mpcd_trainer_comm_init_loopback(self._tr, n, r, key), "mpcd_trainer_comm_init_loopback")
            self.world = (r, n)
            return self
        import torch.distributed as dist
        from .distributed import world
        r, n = world(group)
        if n > 1:
            uid = (ctypes.c_uint8 * N.MPCD_COMM_ID_BYTES)()
            if r == 0:
                N.check(self._lib.mpcd_comm_unique_id(uid), "mpcd_comm_unique_id")
            obj = [bytes(uid)]
            dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
            uid = (ctypes.c_uint8 * N.MPCD_COMM_ID_BYTES).from_buffer_copy(obj[0])
            N.check(self._lib.mpcd_trainer_comm_init(self._tr, n, r, uid), "mpcd_trainer_comm_init")
        self.world = (r, n)
        return self

    def close(self):
        if getattr(self, "_tr", None) and self._tr.value:
            self._lib.mpcd_trainer_destroy(self._tr)
            self._tr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- the reference's random draws
    def draw(self, batch, shape, generator=None):
        """t, noise, context_mask in p_losses' order (loss(): randint; p_losses: randn_like, rand, bernoulli), all
        from torch's CPU generator. This is the reference's stream only for a batch on the CPU: for a CUDA batch
        the reference draws randint / randn_like on x.device (diffusion_model_base.py:435,466) from the CUDA
        generator and only rand / bernoulli on the CPU; pass t / noise explicitly to reproduce such a run."""
        t = torch.randint(0, self.n_steps, (batch,), generator=generator).long()
        noise = torch.randn(shape, generator=generator)
        mask_shape = torch.rand(batch, 1, generator=generator)
        mask = torch.bernoulli(torch.zeros_like(mask_shape) + self.drop_prob, generator=generator)
        return t, noise, mask

    def _run(self, x, context, t, noise, context_mask, update):
        B = x.shape[0]
        if t is None or noise is None or context_mask is None:
            t0, n0, m0 = self.draw(B, tuple(x.shape))
            t = t0 if t is None else t
            noise = n0 if noise is None else noise
            context_mask = m0 if context_mask is None else context_mask
        dev = self.device
        xd = x.detach().to(dev, torch.float32).reshape(B, -1).contiguous()
        cd = context.detach().to(dev, torch.float32).reshape(B, -1).contiguous()
        td = t.detach().to(dev, torch.int64).reshape(B).contiguous()
        nd = noise.detach().to(dev, torch.float32).reshape(B, -1).contiguous()
        md = context_mask.detach().to(dev, torch.float32).reshape(B).contiguous()
        if xd.shape[1] != self.spec.horizon * self.spec.state_dim or cd.shape[1] != self.spec.context_dim:
            raise ValueError("x must be [B, H, d] and context [B, C] of the net's spec")
        if int(td.min()) < 0 or int(td.max()) >= self.n_steps:
            raise ValueError(f"t must lie in [0, {self.n_steps})")
        loss = ctypes.c_double()
        stream = torch.cuda.current_stream(dev).cuda_stream
        N.check(self._lib.mpcd_trainer_step(self._tr, ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(cd.data_ptr()),
                                            ctypes.c_void_p(td.data_ptr()), ctypes.c_void_p(nd.data_ptr()),
                                            ctypes.c_void_p(md.data_ptr()), B, 1 if update else 0, ctypes.byref(loss),
                                            ctypes.c_void_p(stream)), "mpcd_trainer_step")
        return loss.value

    def loss(self, x, context, t=None, noise=None, context_mask=None):
        """GaussianDiffusionModel.loss: p_losses' mean((eps(x_noisy, t, context, mask) - noise)^2), no update."""
        return self._run(x, context, t, noise, context_mask, False)

    def train_step(self, x, context, t=None, noise=None, context_mask=None):
        """One optimisation step: loss, backward, Adam step, EMA update (trainer.py:284-308); returns the loss."""
        return self._run(x, context, t, noise, context_mask, True)

    def state_dict(self, which="params"):
        """{name: tensor} of the model ("params"), the EMA model ("ema"), the last gradients ("grads") or the
        Adam moments ("exp_avg", "exp_avg_sq"), in the net's state_dict names."""
        out = torch.empty(self.n_params, dtype=torch.float32)
        N.check(self._lib.mpcd_trainer_params(self._tr, WHICH[which], ctypes.c_void_p(out.data_ptr()), self.n_params),
                "mpcd_trainer_params")
        sd, o = {}, 0
        for name, shp in self.param_spec:
            n = 1
            for s in shp:
                n *= s
            sd[name] = out[o:o + n].reshape(shp).clone()
            o += n
        return sd
