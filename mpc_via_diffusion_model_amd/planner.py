"""Diffusion-MPC planner: the reference's operator API over the MI355X HIP kernels.

Drop-in for the control-loop body of scripts/inference/Diffusion_MPC_Inference.py:191-289 and
Cart_Diffusion_inference.py:405-512:

  reference                                             here
  GaussianDiffusionModel(model=..., ...) + load_state_dict  DiffusionMPC.from_state_dict(sd, spec)
  dataset.normalize_condition(x0)                        DiffusionMPC.normalize_condition(x0)
  model.run_CFG(context, hard_conds, w, n_samples, horizon, return_chain, sample_fn, n_wo)
                                                         DiffusionMPC.run_CFG(...)   (same signature)
  dataset.unnormalize_states(chain)                      DiffusionMPC.unnormalize_states(x)
  calMPCCost / MPC objective per sample, argmin          DiffusionMPC.mpc_step(x0, system, n_samples)
  (no reference name)                                    DiffusionMPC.sample_trajectories(...)

All compute runs in libmpcd.so (HIP, gfx950); torch supplies device memory, the current stream and
torch.distributed. There is no CPU fallback: a missing library or a failing call raises.
"""
import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _native as N
from . import distributed as D
from . import schedule as S
from .systems import System

_STEP_CONTEXT = object()  # _args placeholder: mpcd_mpc_step normalises x0 into the context itself
_CLIP_RULES = {"chain": N.MPCD_CLIP_CHAIN, "final": N.MPCD_CLIP_FINAL}
_SAMPLERS = {"ddpm_cfg": N.MPCD_DDPM_CFG, "ddpm_cart_pole_sample_fn": N.MPCD_DDPM_CFG,
             "ddim_cfg": N.MPCD_DDIM_CFG, "ddim": N.MPCD_DDIM, "ddim_sample": N.MPCD_DDIM}


def philox_noise(n_cand, n_slices, flat, seed=0, global_offset=0, device=None):
    """The samplers' in-kernel noise for candidates [global_offset, global_offset + n_cand) as a device
    tensor [n_slices, n_cand, flat] (slice 0 = x_T, slice k = denoise step k's draw): feeding it back as
    `noise` replays a Philox run in injected-noise mode (mpcd_philox_noise)."""
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    out = torch.empty((int(n_slices), int(n_cand), int(flat)), dtype=torch.float32, device=dev)
    N.check(N.lib().mpcd_philox_noise(int(seed) & 0xFFFFFFFFFFFFFFFF, int(global_offset), int(n_cand), int(n_slices),
                                      int(flat), ctypes.c_void_p(out.data_ptr()),
                                      ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "mpcd_philox_noise")
    return out


def force_unet_tiling(conv=-1, block=-1):
    """Process-wide U-Net tiling override (mpcd_unet_force_tiling): conv = candidate index for every conv
    (-1: measured), block = fused-block candidate (-1: measured, -2: never fuse)."""
    N.check(N.lib().mpcd_unet_force_tiling(int(conv), int(block)), "mpcd_unet_force_tiling")


UNET_PATHS = {"auto": 0, "layered": 1, "fused": 2}


def force_unet_path(path="auto"):
    """Process-wide U-Net execution form (mpcd_unet_force_path): "auto" (the whole-network fused launch where
    it applies), "layered" (one launch per conv) or "fused" (error where it does not apply)."""
    N.check(N.lib().mpcd_unet_force_path(UNET_PATHS[path]), "mpcd_unet_force_path")


MLP_LAYOUTS = {"auto": -1, "32x8": 0, "16x8": 1, "16x4": 2, "rw32": 3, "rw16": 4}


def force_mlp_layout(layout="auto"):
    """Process-wide MLP sampler workgroup layout (mpcd_mlp_force_layout): "auto" (by batch size), "32x8",
    "16x8" or "16x4" (rows x waves per workgroup), "rw32" / "rw16" (4 waves, resident 128-wide weights)."""
    N.check(N.lib().mpcd_mlp_force_layout(MLP_LAYOUTS[layout]), "mpcd_mlp_force_layout")


@dataclass
class NetSpec:
    """Architecture of the noise-net (temporal_unet.py constructor arguments)."""
    kind: str                 # "mlp" (build-defined CFG MLP) or "unet" (ConditionedTemporalUnet / TemporalUnet)
    state_dim: int            # d
    horizon: int              # H
    context_dim: int          # C (0: TemporalUnet with conditioning None)
    base_dim: int = 32        # unet_input_dim
    dim_mults: tuple = (1, 2, 4)
    time_emb_dim: int = 32
    cfg: bool = True          # 4-arg net with the CFG context mask
    # GEMM numerics (include/mpcd.h mpcd_dtype): "f32" exact fp32 MFMA; "f32x3" fp32-accurate split-bf16
    # MFMA (MLP: shared or no context; UNet: any); "f16" fp16 operands / fp32 accumulate (UNet, cfg 5); "f16x2"
    # two-term fp16 MFMA - NOT fp32 arithmetic: 22-bit operands in the fp16 range (MLP: the CFG-DDPM sampler / eps
    # forward at H*d 32 or 64 with a shared context; U-Net: the fused CFG-DDPM program; the other cases of such a
    # net run its f32x3 kernels). A call that leaves the fp16 range (NaN in the chain) is re-run in f32x3.
    dtype: str = "f32"

    def desc(self):
        d = N.NetDesc()
        d.kind = N.MPCD_NET_MLP if self.kind == "mlp" else N.MPCD_NET_UNET
        d.state_dim, d.horizon, d.context_dim = self.state_dim, self.horizon, self.context_dim
        d.base_dim, d.n_mults = self.base_dim, len(self.dim_mults)
        for i, m in enumerate(self.dim_mults):
            d.mults[i] = m
        d.time_emb_dim = self.time_emb_dim
        d.cfg_masked = 1 if self.cfg else 0
        dtypes = {"f32": N.MPCD_F32, "f16": N.MPCD_F16, "f32x3": N.MPCD_F32X3, "f16x2": N.MPCD_F16X2}
        if self.dtype not in dtypes:
            raise ValueError(f"dtype {self.dtype!r}: use one of {sorted(dtypes)}")
        d.dtype = dtypes[self.dtype]
        return d


@dataclass
class MPCResult:
    u0: np.ndarray          # [d] applied action, unnormalised
    u_best: np.ndarray      # [H, d] winning trajectory, unnormalised
    best_cost: float
    best_index: int         # global candidate index
    costs: torch.Tensor     # [B_total] fp64 on device (all ranks' candidates)
    u_norm: torch.Tensor    # [B_local, H, d] this rank's normalised samples
    flags: int = 0          # mpcd_last_step_flags bits (native step): 1 clipped, 2 NaN in the samples


@dataclass
class ClosedLoopResult:
    x: np.ndarray           # [M, T+1, n_x] plant states (fp64), x[:, 0] = the initial states
    u: np.ndarray           # [M, T, n_u] applied actions (unnormalised, rounded as requested)
    cost: np.ndarray        # [M, T] cost of the selected candidate at each step
    index: np.ndarray       # [M, T] global index of the selected candidate in that step's batch


class DiffusionMPC:
    def __init__(self, spec, params, tables=None, variance_schedule="exponential", n_diffusion_steps=100,
                 device=None, context_limits=None, action_limits=None):
        """params: dict name -> tensor (module state_dict keys, no "model." prefix) in any order.
        tables: dict of the 12 diffusion buffers (e.g. from a checkpoint) or None to compute them."""
        self.spec = spec
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.n_steps = n_diffusion_steps if tables is None else int(tables["betas"].numel())
        self.tables = tables if tables is not None else S.tables(variance_schedule, n_diffusion_steps)
        if not S.is_finite(self.tables):
            raise ValueError(f"{variance_schedule} schedule with N={self.n_steps} is not finite "
                             "(the reference would produce NaN; use 'cosine' or another N)")
        c_lo, c_hi = context_limits if context_limits is not None else (-np.ones(spec.context_dim),
                                                                        np.ones(spec.context_dim))
        a_lo, a_hi = action_limits if action_limits is not None else (-np.ones(spec.state_dim),
                                                                      np.ones(spec.state_dim))
        self.ctx_min = np.ascontiguousarray(c_lo, dtype=np.float32)
        self.ctx_max = np.ascontiguousarray(c_hi, dtype=np.float32)
        self.act_min = np.ascontiguousarray(a_lo, dtype=np.float32)
        self.act_max = np.ascontiguousarray(a_hi, dtype=np.float32)
        self._lib = N.lib()
        self._ctx = ctypes.c_void_p()
        N.check(self._lib.mpcd_create(self.device.index, ctypes.byref(self._ctx)), "mpcd_create")
        self._desc = spec.desc()
        self.param_spec = N.param_spec(self._desc)
        blob = torch.cat([params[n].detach().to("cpu", torch.float32).reshape(-1) for n, _ in self.param_spec])
        for n, shp in self.param_spec:
            if tuple(params[n].shape) != shp:
                raise ValueError(f"{n}: shape {tuple(params[n].shape)} != {shp}")
        blob = blob.contiguous()
        N.check(self._lib.mpcd_load_net(self._ctx, ctypes.byref(self._desc), ctypes.c_void_p(blob.data_ptr()),
                                        blob.numel()), "mpcd_load_net")
        tab = S.pack(self.tables)
        std = S.posterior_std(self.tables).contiguous()
        N.check(self._lib.mpcd_set_schedule(self._ctx, ctypes.c_void_p(tab.data_ptr()), self.n_steps,
                                            ctypes.c_void_p(std.data_ptr())), "mpcd_set_schedule")
        # DDPM with clip_denoised ends with x = coef1[0]*clamp(x0) + coef2[0]*x: if coef2[0] == 0 and
        # |coef1[0]| <= 1 + 1e-4 the clip flag over the FINAL samples is provably 0 (clip_rule="final";
        # the reference's chain-wide rule still sees x_T and is computed).
        c1, c2 = float(self.tables["posterior_mean_coef1"][0]), float(self.tables["posterior_mean_coef2"][0])
        self.ddpm_final_in_range = c2 == 0.0 and abs(c1) <= np.float32(1 + 1e-4)
        self._flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._best = torch.zeros(2, dtype=torch.float64, device=self.device)  # mpcd_best {double, int64}

    # ------------------------------------------------------------------ construction helpers
    @classmethod
    def from_state_dict(cls, state_dict, spec, **kw):
        """Reference checkpoint layout: "model.<param>" + the 12 schedule buffers (weights-only load)."""
        has_prefix = any(k.startswith("model.") for k in state_dict)
        params = {k[6:] if has_prefix and k.startswith("model.") else k: v for k, v in state_dict.items()}
        tables = None
        if all(k in state_dict for k in S.TABLE_ORDER):
            tables = {k: state_dict[k].detach().cpu().to(torch.float32) for k in S.TABLE_ORDER}
        return cls(spec, params, tables=tables, **kw)

    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            self._lib.mpcd_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ normalisation (A12)
    def normalize_condition(self, x0):
        """LimitsNormalizer.normalize of the fp64 state (normalization.py:149-154), cast to fp32 as the
        net's c_emb.float() does (temporal_unet.py:314). Host-side: C values per control step."""
        x = np.asarray(x0, dtype=np.float64)
        mn = self.ctx_min.astype(np.float64)
        den = (self.ctx_max - self.ctx_min).astype(np.float64)  # fp32 subtraction, then promoted
        return (2 * ((x - mn) / den) - 1).astype(np.float32)

    def unnormalize_states(self, x, clip_flag=None):
        """LimitsNormalizer.unnormalize on device (normalization.py:156-167), global clip rule."""
        x = x.contiguous()
        out = torch.empty_like(x)
        d = x.shape[-1]
        flag_ptr = ctypes.c_void_p(clip_flag.data_ptr()) if clip_flag is not None else None
        N.check(self._lib.mpcd_unnormalize(self._ctx, ctypes.c_void_p(x.data_ptr()), x.numel() // d, d,
                                           self.act_min.ctypes.data, self.act_max.ctypes.data, flag_ptr,
                                           ctypes.c_void_p(out.data_ptr()), self._stream()), "mpcd_unnormalize")
        return out

    # ------------------------------------------------------------------ sampling (A2-A11)
    def _system_desc(self, system):
        """system.desc() (a ctypes struct), rebuilt only when the system's fields change: a control loop calls
        mpc_step with the same system every step."""
        key = (system.system, system.cost_kind, system.n_x, system.n_u, tuple(system.params), tuple(system.Q),
               tuple(system.R), tuple(system.P), tuple(system.x_ref or ()))
        c = getattr(self, "_desc_cache", None)
        if c is None or c[0] != key:
            c = self._desc_cache = (key, system.desc())
        return c[1]

    def _stream(self):
        # the raw handle of the device's current stream (torch.cuda.current_stream(device).cuda_stream without
        # building a Stream object: this runs once per control step on the host path)
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        if raw is not None:
            return ctypes.c_void_p(raw(self.device.index))
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _sampler_id(self, sample_fn):
        name = sample_fn if isinstance(sample_fn, str) else getattr(sample_fn, "__name__", str(sample_fn))
        if name not in _SAMPLERS:
            raise ValueError(f"unsupported sample_fn {name!r}; use one of {sorted(_SAMPLERS)}")
        return _SAMPLERS[name]

    def _args(self, sampler, batch, context, w, n_wo_noise, ddim_steps, clamp_x0, seed, global_offset, noise,
              x_out, chain, absmax=None):
        a = N.SampleArgs()
        if self.spec.context_dim > 0 and context is not _STEP_CONTEXT:
            if context is None:
                raise ValueError("this net needs a context")
            a.context = context.data_ptr()
            a.context_shared = 1 if context.shape[0] == 1 else 0
            if not a.context_shared and context.shape[0] != batch:
                raise ValueError(f"context rows {context.shape[0]} must be 1 or n_samples={batch}")
        a.sampler = sampler
        a.batch = batch
        a.w = float(w)
        a.n_wo_noise = int(n_wo_noise)
        a.ddim_steps = int(ddim_steps or 0)
        a.clamp_x0 = 1 if clamp_x0 else 0
        if sampler != N.MPCD_DDPM_CFG:
            times = S.ddim_times(self.n_steps, ddim_steps or None)
            self._times = (ctypes.c_int32 * len(times))(*times)
            a.ddim_times = ctypes.cast(self._times, ctypes.POINTER(ctypes.c_int32))
            a.n_ddim_times = len(times)
        a.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        a.global_offset = int(global_offset)
        a.noise = noise.data_ptr() if noise is not None else None
        a.x_out = x_out.data_ptr()
        a.chain_out = chain.data_ptr() if chain is not None else None
        a.chain_absmax = absmax.data_ptr() if absmax is not None else None
        return a

    def n_denoise_steps(self, sample_fn="ddpm_cfg", n_wo_noise=0, ddim_steps=None):
        a = N.SampleArgs()
        a.sampler = self._sampler_id(sample_fn)
        a.n_wo_noise = n_wo_noise
        a.ddim_steps = int(ddim_steps or 0)
        if a.sampler != N.MPCD_DDPM_CFG:
            times = S.ddim_times(self.n_steps, ddim_steps or None)
            self._times = (ctypes.c_int32 * len(times))(*times)
            a.ddim_times = ctypes.cast(self._times, ctypes.POINTER(ctypes.c_int32))
            a.n_ddim_times = len(times)
        n = ctypes.c_int32()
        N.check(self._lib.mpcd_sample_steps(self._ctx, ctypes.byref(a), ctypes.byref(n)), "mpcd_sample_steps")
        return n.value

    def sample_trajectories(self, context=None, n_samples=1, horizon=None, w=0.01, sample_fn="ddpm_cfg",
                            n_wo_noise=0, ddim_steps=None, clamp_x0=False, seed=0, global_offset=0, noise=None,
                            return_chain=False, out=None, absmax_out=None):
        """Normalised candidate trajectories [B, H, d] (or the chain [S+1, B, H, d]).
        context: [1, C] (shared) or [B, C] normalised fp32; noise: optional injected [S+1, B, H, d].
        absmax_out: optional fp32 [B] device tensor <- per candidate max |x| over the whole chain
        (x_T .. x_0; NaN if any NaN): the input of the reference's chain-wide clip test without
        materialising the chain."""
        H = horizon or self.spec.horizon
        if H != self.spec.horizon:
            raise ValueError(f"net was built for horizon {self.spec.horizon}")
        sampler = self._sampler_id(sample_fn)
        B = int(n_samples)
        d = self.spec.state_dim
        if context is not None:
            context = torch.as_tensor(context, dtype=torch.float32)
            if context.dim() == 1:
                context = context[None]
            context = context.to(self.device).contiguous()
        steps = self.n_denoise_steps(sample_fn, n_wo_noise, ddim_steps)
        if noise is not None:
            noise = noise.to(self.device, torch.float32).contiguous()
            if tuple(noise.shape) != (steps + 1, B, H, d):
                raise ValueError(f"noise must be [{steps + 1}, {B}, {H}, {d}], got {tuple(noise.shape)}")
        x = out if out is not None else torch.empty((B, H, d), dtype=torch.float32, device=self.device)
        chain = torch.empty((steps + 1, B, H, d), dtype=torch.float32, device=self.device) if return_chain else None
        if absmax_out is not None and (absmax_out.dtype != torch.float32 or absmax_out.numel() != B
                                       or absmax_out.device != self.device or not absmax_out.is_contiguous()):
            raise ValueError(f"absmax_out must be a contiguous fp32 [{B}] tensor on {self.device}")
        # f16x2 numerics compute in the fp16 range: ask for the chain maxima (a NaN there = a value left the range),
        # check them (one synchronisation) and re-run the call with the net's split-bf16 programs if so
        guard = self.spec.dtype == "f16x2"
        amax = absmax_out
        if guard and amax is None:
            amax = torch.empty(B, dtype=torch.float32, device=self.device)
        a = self._args(sampler, B, context, w, n_wo_noise, ddim_steps, clamp_x0, seed, global_offset, noise, x, chain,
                       amax)
        N.check(self._lib.mpcd_sample(self._ctx, ctypes.byref(a), self._stream()), "mpcd_sample")
        self.last_f32x3_rerun = False
        if guard and bool(torch.isnan(amax).any()):
            N.check(self._lib.mpcd_force_f32x3(self._ctx, 1), "mpcd_force_f32x3")
            try:
                N.check(self._lib.mpcd_sample(self._ctx, ctypes.byref(a), self._stream()), "mpcd_sample (f32x3 re-run)")
            finally:
                N.check(self._lib.mpcd_force_f32x3(self._ctx, 0), "mpcd_force_f32x3")
            self.last_f32x3_rerun = True
        return chain if return_chain else x

    def run_CFG(self, context=None, hard_conds=None, context_weight=0.1, n_samples=1, horizon=8,
                return_chain=False, sample_fn="ddpm_cart_pole_sample_fn", n_diffusion_steps_without_noise=0,
                noise=None, seed=0, **_unused):
        """GaussianDiffusionModel.run_CFG (diffusion_model_base.py:394-418): chain [S+1, B, H, d] or
        the final [B, H, d], normalised. hard_conds is ignored as in the reference (commented out there)."""
        return self.sample_trajectories(context, n_samples, horizon, context_weight, sample_fn,
                                        n_diffusion_steps_without_noise, noise=noise, seed=seed,
                                        return_chain=return_chain)

    def eps(self, x, t, context=None):
        """Noise-net forward(s) at time t: (eps_cond, eps_uncond) for a CFG net, (eps, None) otherwise."""
        x = x.to(self.device, torch.float32).contiguous()
        B = x.shape[0]
        if context is not None:
            context = torch.as_tensor(context, dtype=torch.float32).to(self.device).contiguous()
            if context.dim() == 1:
                context = context[None]
        ec = torch.empty_like(x)
        eu = torch.empty_like(x) if self.spec.cfg else None
        N.check(self._lib.mpcd_eps(self._ctx, ctypes.c_void_p(x.data_ptr()), int(t),
                                   ctypes.c_void_p(context.data_ptr()) if context is not None else None,
                                   1 if context is not None and context.shape[0] == 1 else 0, B,
                                   ctypes.c_void_p(ec.data_ptr()), ctypes.c_void_p(eu.data_ptr()) if eu is not None else None,
                                   self._stream()), "mpcd_eps")
        return ec, eu

    def unet_form(self, sample_fn="ddpm_cfg"):
        """The U-Net execution form an mpc_step / sample call with this sampler takes (mpcd_unet_form):
        {"fused": bool, "planes": 0 | 1 | 3, "rows_per_workgroup": R, "waves_per_workgroup": W} - the kernel
        bench.py names."""
        out = (ctypes.c_int32 * 4)()
        N.check(self._lib.mpcd_unet_form(self._ctx, self._sampler_id(sample_fn), out), "mpcd_unet_form")
        return {"fused": bool(out[0]), "planes": int(out[1]), "rows_per_workgroup": int(out[2]),
                "waves_per_workgroup": int(out[3])}

    def mlp_layout(self, n_samples):
        """The MLP sampler layout ("32x8", "16x8", "16x4", "rw32", "rw16") a sample call of n_samples runs."""
        out = ctypes.c_int32()
        with torch.cuda.device(self.device):  # the library decides on the current device's CU count
            N.check(self._lib.mpcd_mlp_layout(int(n_samples), int(self.spec.cfg), ctypes.byref(out)), "mpcd_mlp_layout")
        return {v: k for k, v in MLP_LAYOUTS.items()}[out.value]

    def mlp_form(self, n_samples, sample_fn="ddpm_cfg"):
        """The MLP kernel a shared-context sample call of n_samples runs (mpcd_mlp_form): {"kernel": "f32" | "x3" |
        "h2", "layout": the bf16x3 layout name or None, "rows_per_workgroup": 32 | 16}."""
        out = (ctypes.c_int32 * 3)()
        N.check(self._lib.mpcd_mlp_form(self._ctx, self._sampler_id(sample_fn), int(n_samples), out), "mpcd_mlp_form")
        lay = {v: k for k, v in MLP_LAYOUTS.items()}.get(out[1]) if out[1] >= 0 else None
        return {"kernel": ("f32", "x3", "h2")[out[0]], "layout": lay, "rows_per_workgroup": int(out[2])}

    def last_sample_ms(self):
        ms = ctypes.c_float()
        N.check(self._lib.mpcd_last_sample_ms(self._ctx, ctypes.byref(ms)), "mpcd_last_sample_ms")
        return ms.value

    def sample_ms_mean(self, n):
        """Mean sampler-kernel time (HIP events) over the last n sample calls (n <= 256), read once after a loop."""
        ms = ctypes.c_float()
        N.check(self._lib.mpcd_sample_ms_mean(self._ctx, int(n), ctypes.byref(ms)), "mpcd_sample_ms_mean")
        return ms.value

    # ------------------------------------------------------------------ rollout / cost / selection (A13-A15)
    def rollout_cost(self, system: System, x0, u_norm, clip_flag=None):
        """fp64 cost per candidate [B] on device."""
        B, H, d = u_norm.shape
        if d != system.n_u:
            raise ValueError(f"system {system.name} has {system.n_u} inputs, samples have {d}")
        x0 = np.ascontiguousarray(x0, dtype=np.float64)
        cost = torch.empty(B, dtype=torch.float64, device=self.device)
        desc = system.desc()
        flag_ptr = ctypes.c_void_p(clip_flag.data_ptr()) if clip_flag is not None else None
        N.check(self._lib.mpcd_rollout_cost(self._ctx, ctypes.byref(desc), x0.ctypes.data,
                                            ctypes.c_void_p(u_norm.contiguous().data_ptr()), self.act_min.ctypes.data,
                                            self.act_max.ctypes.data, B, H, flag_ptr, ctypes.c_void_p(cost.data_ptr()),
                                            self._stream()), "mpcd_rollout_cost")
        return cost

    def clip_flag(self, x):
        flag = torch.empty(1, dtype=torch.int32, device=self.device)
        N.check(self._lib.mpcd_clip_flag(self._ctx, ctypes.c_void_p(x.data_ptr()), x.numel(),
                                         ctypes.c_void_p(flag.data_ptr()), self._stream()), "mpcd_clip_flag")
        return flag

    def argmin(self, cost, index_offset=0):
        """Device argmin (NaN = +inf, lowest index on ties) -> (index, cost); syncs the stream."""
        N.check(self._lib.mpcd_argmin(self._ctx, ctypes.c_void_p(cost.data_ptr()), cost.numel(), index_offset,
                                      ctypes.c_void_p(self._best.data_ptr()), self._stream()), "mpcd_argmin")
        host = self._best.cpu()
        return int(host.view(torch.int64)[1]), float(host[0])

    def closed_loop(self, x0_states, system: System, iterations, n_samples=1, w=0.01, sample_fn="ddpm_cfg",
                    n_wo_noise=0, ddim_steps=None, clamp_x0=False, select="argmin", decimals=4, seed=0, noise=None,
                    clip_rule="chain"):
        """Closed-loop diffusion MPC for M plant states at once, resident on the device.
        The reference runs one initial state at a time on the host (Cart_Diffusion_inference.py:405-512:
        normalize_condition -> run_CFG -> unnormalize -> u0 = round(u[0], 4) -> x = f(x, u0), repeated
        ITERATIONS times per initial state). Here every iteration is: per-state contexts
        (mpcd_normalize_states), n_samples candidates per state in one sampler launch, per-state clip flags,
        rollout + cost from each state's own x, and mpcd_control_step (per-state selection, u0, plant step);
        nothing returns to the host until the end. select: "argmin" (lowest cost) or "first" (candidate 0 of
        each group: the reference scripts with n_samples = 1). Per-state contexts use the exact-f32 MLP
        kernel (the split-bf16 one needs a shared context). noise: optional callable it -> injected sampler
        noise [S+1, M*n_samples, H, d] (parity tests); default in-kernel Philox keyed by (seed + it).
        clip_rule: "chain" (the reference: run_CFG(return_chain=True) then unnormalize_states of the whole
        chain, so each state's clip test also sees its x_T) or "final" (the final samples only)."""
        if select not in ("argmin", "first"):
            raise ValueError("select must be 'argmin' or 'first'")
        if clip_rule not in _CLIP_RULES:
            raise ValueError(f"clip_rule must be one of {sorted(_CLIP_RULES)}")
        x0 = np.ascontiguousarray(np.atleast_2d(np.asarray(x0_states, dtype=np.float64)))
        M, nx = x0.shape
        if nx != system.n_x or system.n_u != self.spec.state_dim:
            raise ValueError(f"system {system.name}: n_x={system.n_x}, n_u={system.n_u}; states have {nx} columns, "
                             f"the net samples {self.spec.state_dim} actions")
        if self.spec.context_dim != nx:
            raise ValueError(f"closed loop conditions on the plant state: context_dim {self.spec.context_dim} != n_x {nx}")
        T, n, H, d = int(iterations), int(n_samples), self.spec.horizon, self.spec.state_dim
        B, dev, st = M * n, self.device, self._stream()
        desc = system.desc()
        x = torch.from_numpy(x0).to(dev)
        xs = torch.empty((T + 1, M, nx), dtype=torch.float64, device=dev)
        us = torch.empty((T, M, d), dtype=torch.float64, device=dev)
        cs = torch.empty((T, M), dtype=torch.float64, device=dev)
        ix = torch.empty((T, M), dtype=torch.int64, device=dev)
        ctx = torch.empty((M, nx), dtype=torch.float32, device=dev)
        flags = torch.empty(M, dtype=torch.int32, device=dev)
        cost = torch.empty(B, dtype=torch.float64, device=dev)
        u_norm = torch.empty((B, H, d), dtype=torch.float32, device=dev)
        absmax = torch.empty(B, dtype=torch.float32, device=dev) if clip_rule == "chain" else None
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        xs[0] = x
        for it in range(T):
            N.check(self._lib.mpcd_normalize_states(self._ctx, ptr(x), M, nx, self.ctx_min.ctypes.data,
                                                    self.ctx_max.ctypes.data, ptr(ctx), st), "mpcd_normalize_states")
            self.sample_trajectories(ctx.repeat_interleave(n, dim=0), B, H, w, sample_fn, n_wo_noise, ddim_steps,
                                     clamp_x0, seed + it, 0, None if noise is None else noise(it), False, out=u_norm,
                                     absmax_out=absmax)
            if absmax is not None:  # each state's flag over its candidates' chains
                N.check(self._lib.mpcd_clip_flags(self._ctx, ptr(absmax), M, n, ptr(flags), st), "mpcd_clip_flags")
            else:
                N.check(self._lib.mpcd_clip_flags(self._ctx, ptr(u_norm), M, n * H * d, ptr(flags), st), "mpcd_clip_flags")
            N.check(self._lib.mpcd_rollout_cost_grouped(self._ctx, ctypes.byref(desc), ptr(x), n, ptr(u_norm),
                                                        self.act_min.ctypes.data, self.act_max.ctypes.data, B, H,
                                                        ptr(flags), ptr(cost), st), "mpcd_rollout_cost_grouped")
            N.check(self._lib.mpcd_control_step(self._ctx, ctypes.byref(desc), ptr(x), M, n, ptr(u_norm), H, ptr(cost),
                                                self.act_min.ctypes.data, self.act_max.ctypes.data, ptr(flags),
                                                1 if select == "first" else 0, -1 if decimals is None else int(decimals),
                                                ptr(us[it]), ptr(ix[it]), ptr(cs[it]), st), "mpcd_control_step")
            xs[it + 1] = x
        return ClosedLoopResult(x=xs.transpose(0, 1).cpu().numpy(), u=us.transpose(0, 1).cpu().numpy(),
                                cost=cs.t().cpu().numpy(), index=ix.t().cpu().numpy())

    def mpc_step(self, x0, system: System, n_samples, w=0.01, sample_fn="ddpm_cfg", n_wo_noise=0, ddim_steps=None,
                 clamp_x0=False, seed=0, noise=None, group=None, comm=None, native=None, clip_rule="chain"):
        """One control step: sample n_samples candidates on this rank (weak scaling: every rank adds
        n_samples), roll out + cost them, all-gather costs, pick the global argmin, broadcast it.
        comm: a distributed.NativeComm (the exchange inside libmpcd.so over RCCL) or None
        (torch.distributed collectives on `group`).
        native: run the whole step as one mpcd_mpc_step call (default whenever the library can do the
        exchange itself: a NativeComm, or a single rank); False = the step composed from the separate
        entry points (sample, clip flag, rollout, select), kept as the reference composition.
        clip_rule: which tensor LimitsNormalizer's global clip test runs over. "chain" (default) = the
        reference scripts, which call run_CFG(return_chain=True) and unnormalise the whole chain
        (Cart_Diffusion_inference.py:450-463, Diffusion_MPC_Inference.py:232-247), so x_T ~ N(0, 1) is in
        the test; "final" = the final samples only (proven 0 for DDPM when the last posterior mean cannot
        leave [-1, 1], then no reduction is run)."""
        if clip_rule not in _CLIP_RULES:
            raise ValueError(f"clip_rule must be one of {sorted(_CLIP_RULES)}")
        if comm is not None:
            rank, size = comm.rank, comm.size
        else:
            rank, size = D.world(group)
        if native is None:
            native = comm is not None or size == 1
        if native:
            if size > 1 and comm is None:
                raise ValueError("native mpc_step on several ranks needs a NativeComm")
            return self._mpc_step_native(x0, system, n_samples, w, sample_fn, n_wo_noise, ddim_steps, clamp_x0, seed,
                                         noise, comm, clip_rule)
        offset = rank * n_samples
        ctx = torch.from_numpy(self.normalize_condition(x0)[None]) if self.spec.context_dim > 0 else None
        absmax = torch.empty(n_samples, dtype=torch.float32, device=self.device) if clip_rule == "chain" else None
        u_norm = self.sample_trajectories(ctx, n_samples, self.spec.horizon, w, sample_fn, n_wo_noise, ddim_steps,
                                          clamp_x0, seed, offset, noise, absmax_out=absmax)
        # LimitsNormalizer's clip flag is global over the whole batch: this rank's own code, the max over
        # ranks (mpcd_clip_flag codes: 1 = clip, 2 = NaN seen), or provably zero (final-samples rule,
        # DDPM whose last posterior mean stays in range) -> no exchange
        sampler = self._sampler_id(sample_fn)
        if clip_rule == "final" and sampler == N.MPCD_DDPM_CFG and self.ddpm_final_in_range:
            flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        else:
            flag = self.clip_flag(absmax if absmax is not None else u_norm)
            if size > 1:
                flag = comm.any_flag(flag) if comm else D.any_flag(flag, group)
        cost_local = self.rollout_cost(system, x0, u_norm, flag)
        if comm is not None:
            idx, best, row, costs = comm.select(cost_local, u_norm)
        else:
            idx, best, row, costs = D.select(cost_local, u_norm, self.argmin, group)
        u_best = self.unnormalize_states(row[None], flag)[0]
        u_host = u_best.cpu().numpy()
        return MPCResult(u0=u_host[0].copy(), u_best=u_host, best_cost=best, best_index=idx, costs=costs,
                         u_norm=u_norm)

    def _mpc_step_native(self, x0, system, n_samples, w, sample_fn, n_wo_noise, ddim_steps, clamp_x0, seed, noise,
                         comm, clip_rule="chain"):
        """mpc_step as one libmpcd call (mpcd_mpc_step): one H2D copy of the context row, the kernels,
        the result block {best, u_best} written to pinned host memory by the selecting workgroup (one rank) or one
        D2H copy + stream synchronisation (with a communicator)."""
        size, rank = (comm.size, comm.rank) if comm is not None else (1, 0)
        B, H, d = int(n_samples), self.spec.horizon, self.spec.state_dim
        if d != system.n_u:
            raise ValueError(f"system {system.name} has {system.n_u} inputs, samples have {d}")
        sampler = self._sampler_id(sample_fn)
        if noise is not None:
            steps = self.n_denoise_steps(sample_fn, n_wo_noise, ddim_steps)
            noise = noise.to(self.device, torch.float32).contiguous()
            if tuple(noise.shape) != (steps + 1, B, H, d):
                raise ValueError(f"noise must be [{steps + 1}, {B}, {H}, {d}], got {tuple(noise.shape)}")
        u_norm = torch.empty((B, H, d), dtype=torch.float32, device=self.device)
        cost = torch.empty(B, dtype=torch.float64, device=self.device)
        costs = torch.empty(size * B, dtype=torch.float64, device=self.device) if size > 1 else cost
        x0 = np.ascontiguousarray(x0, dtype=np.float64)
        desc = self._system_desc(system)
        # the argument block of a control loop's repeated call is built once and patched per step (x0, seed, the
        # output pointers): the host path between two sampler launches is part of every control step's latency
        key = (id(desc), B, sampler, float(w), int(n_wo_noise), ddim_steps, bool(clamp_x0), clip_rule, size, rank,
               noise is None)
        cache = getattr(self, "_step_args_cache", None)
        if cache is None or cache[0] != key:
            a = N.StepArgs()
            a.sys = ctypes.pointer(desc)
            a.ctx_min, a.ctx_max = self.ctx_min.ctypes.data, self.ctx_max.ctypes.data
            a.act_min, a.act_max = self.act_min.ctypes.data, self.act_max.ctypes.data
            a.sample = self._args(sampler, B, _STEP_CONTEXT, w, n_wo_noise, ddim_steps, clamp_x0, seed, rank * B,
                                  noise, u_norm, None)
            a.clip_rule = _CLIP_RULES[clip_rule]
            if clip_rule == "final" and sampler == N.MPCD_DDPM_CFG and self.ddpm_final_in_range:
                a.clip_rule = N.MPCD_CLIP_NONE
            # (+ the DDIM time list a.sample points into, kept alive with the block)
            cache = self._step_args_cache = (key, a, ctypes.byref(a), desc, N.Best(), ctypes.c_int32(),
                                             getattr(self, "_times", None))
        _, a, a_ref, _, best, fl, _ = cache
        sa = a.sample
        sa.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        sa.x_out = u_norm.data_ptr()
        sa.noise = noise.data_ptr() if noise is not None else None
        a.x0 = x0.__array_interface__["data"][0]
        a.cost_local = cost.data_ptr()
        a.costs_all = costs.data_ptr()
        u_best = np.empty((H, d), dtype=np.float32)
        # MPCD_ENONFINITE (no candidate with a finite cost: NaN / Inf samples) raises MpcdError here
        N.check(self._lib.mpcd_mpc_step(self._ctx, a_ref, ctypes.byref(best), u_best.__array_interface__["data"][0],
                                        self._stream()), "mpcd_mpc_step")
        N.check(self._lib.mpcd_last_step_flags(self._ctx, ctypes.byref(fl)), "mpcd_last_step_flags")
        return MPCResult(u0=u_best[0].copy(), u_best=u_best, best_cost=best.cost, best_index=best.index, costs=costs,
                         u_norm=u_norm, flags=fl.value)
