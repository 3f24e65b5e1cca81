"""ctypes binding of libmpcd.so (include/mpcd.h).

The product path has no fallback: if the library is missing or a call fails, this raises.
torch is imported first so the process has exactly one HIP runtime (torch's libamdhip64.so.7,
which the library's DT_NEEDED entry then resolves to).
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before libmpcd.so)

_HERE = os.path.dirname(os.path.abspath(__file__))
# MPCD_LIB: load an experiment build (build.py variant) instead of the product library
LIB_PATH = os.environ.get("MPCD_LIB") or os.path.join(_HERE, "libmpcd.so")

MPCD_NET_MLP, MPCD_NET_UNET = 1, 2
MPCD_F32, MPCD_F16, MPCD_F32X3, MPCD_F16X2 = 0, 1, 2, 3
MPCD_DDPM_CFG, MPCD_DDIM_CFG, MPCD_DDIM = 0, 1, 2
MPCD_COST_CANONICAL, MPCD_COST_CALMPC = 0, 1
MPCD_COMM_ID_BYTES = 128
MPCD_CLIP_CHAIN, MPCD_CLIP_FINAL, MPCD_CLIP_NONE = 0, 1, 2

_STATUS = {-1: "EINVAL", -2: "EHIP", -3: "ESTATE", -4: "ENOMEM", -5: "EUNSUP", -6: "ENONFINITE"}
MPCD_ENONFINITE = -6
MPCD_STEP_CLIPPED, MPCD_STEP_NAN_SAMPLES, MPCD_STEP_NONFINITE_WINNER, MPCD_STEP_F32X3_RERUN = 1, 2, 4, 8


class NetDesc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("state_dim", ctypes.c_int32), ("horizon", ctypes.c_int32),
                ("context_dim", ctypes.c_int32), ("base_dim", ctypes.c_int32), ("n_mults", ctypes.c_int32),
                ("mults", ctypes.c_int32 * 4), ("time_emb_dim", ctypes.c_int32), ("cfg_masked", ctypes.c_int32),
                ("dtype", ctypes.c_int32)]


class SampleArgs(ctypes.Structure):
    _fields_ = [("context", ctypes.c_void_p), ("context_shared", ctypes.c_int32), ("sampler", ctypes.c_int32),
                ("batch", ctypes.c_int64), ("w", ctypes.c_double), ("n_wo_noise", ctypes.c_int32),
                ("ddim_steps", ctypes.c_int32), ("clamp_x0", ctypes.c_int32), ("n_ddim_times", ctypes.c_int32),
                ("ddim_times", ctypes.POINTER(ctypes.c_int32)), ("seed", ctypes.c_uint64),
                ("global_offset", ctypes.c_int64), ("noise", ctypes.c_void_p), ("x_out", ctypes.c_void_p),
                ("chain_out", ctypes.c_void_p), ("chain_absmax", ctypes.c_void_p)]


class SystemDesc(ctypes.Structure):
    _fields_ = [("system", ctypes.c_int32), ("cost_kind", ctypes.c_int32), ("n_x", ctypes.c_int32),
                ("n_u", ctypes.c_int32), ("params", ctypes.c_double * 24), ("Q", ctypes.c_double * 12),
                ("R", ctypes.c_double * 4), ("P", ctypes.c_double * 12), ("x_ref", ctypes.c_double * 12)]


class Best(ctypes.Structure):
    _fields_ = [("cost", ctypes.c_double), ("index", ctypes.c_int64)]


class StepArgs(ctypes.Structure):
    _fields_ = [("sys", ctypes.POINTER(SystemDesc)), ("x0", ctypes.c_void_p), ("ctx_min", ctypes.c_void_p),
                ("ctx_max", ctypes.c_void_p), ("act_min", ctypes.c_void_p), ("act_max", ctypes.c_void_p),
                ("sample", SampleArgs), ("clip_rule", ctypes.c_int32), ("cost_local", ctypes.c_void_p),
                ("costs_all", ctypes.c_void_p)]


class TrainCfg(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
                ("ema_decay", ctypes.c_float), ("step_start_ema", ctypes.c_int32), ("update_ema_every", ctypes.c_int32)]


EXPORTS = {
    "mpcd_net_param_count": ([ctypes.POINTER(NetDesc), ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)],
                             ctypes.c_int),
    "mpcd_net_param_info": ([ctypes.POINTER(NetDesc), ctypes.c_int32, ctypes.c_char_p, ctypes.c_size_t,
                             ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)], ctypes.c_int),
    "mpcd_create": ([ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "mpcd_destroy": ([ctypes.c_void_p], None),
    "mpcd_last_error": ([], ctypes.c_char_p),
    "mpcd_load_net": ([ctypes.c_void_p, ctypes.POINTER(NetDesc), ctypes.c_void_p, ctypes.c_size_t], ctypes.c_int),
    "mpcd_set_schedule": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p], ctypes.c_int),
    "mpcd_sample_steps": ([ctypes.c_void_p, ctypes.POINTER(SampleArgs), ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "mpcd_sample": ([ctypes.c_void_p, ctypes.POINTER(SampleArgs), ctypes.c_void_p], ctypes.c_int),
    "mpcd_eps": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "mpcd_clip_flag": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p],
                       ctypes.c_int),
    "mpcd_rollout_cost": ([ctypes.c_void_p, ctypes.POINTER(SystemDesc), ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "mpcd_unnormalize": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "mpcd_argmin": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                     ctypes.c_void_p], ctypes.c_int),
    "mpcd_last_sample_ms": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
    "mpcd_sample_ms_mean": ([ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
    "mpcd_clip_flags": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                         ctypes.c_void_p], ctypes.c_int),
    "mpcd_normalize_states": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "mpcd_rollout_cost_grouped": ([ctypes.c_void_p, ctypes.POINTER(SystemDesc), ctypes.c_void_p, ctypes.c_int64,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "mpcd_control_step": ([ctypes.c_void_p, ctypes.POINTER(SystemDesc), ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                           ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "mpcd_comm_unique_id": ([ctypes.c_void_p], ctypes.c_int),
    "mpcd_comm_init": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p], ctypes.c_int),
    "mpcd_philox_noise": ([ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                           ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "mpcd_last_step_flags": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "mpcd_unet_force_tiling": ([ctypes.c_int32, ctypes.c_int32], ctypes.c_int),
    "mpcd_mlp_force_layout": ([ctypes.c_int32], ctypes.c_int),
    "mpcd_force_f32x3": ([ctypes.c_void_p, ctypes.c_int32], ctypes.c_int),
    "mpcd_mlp_layout": ([ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "mpcd_mlp_form": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "mpcd_unet_force_path": ([ctypes.c_int32], ctypes.c_int),
    "mpcd_unet_form": ([ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "mpcd_comm_init_loopback": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64], ctypes.c_int),
    "mpcd_comm_info": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "mpcd_allgather_f32": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p],
                           ctypes.c_int),
    "mpcd_allgather_f64": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p],
                           ctypes.c_int),
    "mpcd_broadcast_f32": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_void_p],
                           ctypes.c_int),
    "mpcd_allreduce_max_i32": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p], ctypes.c_int),
    "mpcd_mpc_step": ([ctypes.c_void_p, ctypes.POINTER(StepArgs), ctypes.POINTER(Best), ctypes.c_void_p,
                       ctypes.c_void_p], ctypes.c_int),
    "mpcd_trainer_create": ([ctypes.POINTER(NetDesc), ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(TrainCfg),
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)],
                            ctypes.c_int),
    "mpcd_trainer_step": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_double),
                           ctypes.c_void_p], ctypes.c_int),
    "mpcd_trainer_params": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t], ctypes.c_int),
    "mpcd_trainer_destroy": ([ctypes.c_void_p], None),
    "mpcd_trainer_comm_init": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p], ctypes.c_int),
    "mpcd_trainer_comm_init_loopback": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64], ctypes.c_int),
    "mpcd_select": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
}

_lib = None


class MpcdError(RuntimeError):
    def __init__(self, msg, status=None):
        super().__init__(msg)
        self.status = status


def lib():
    """Load libmpcd.so (raises if it was not built: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MpcdError(f"{LIB_PATH} is missing: run `python -m mpc_via_diffusion_model_amd.build` "
                            "(the HIP library is required; there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (argt, rest) in EXPORTS.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = rest
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().mpcd_last_error().decode(errors="replace")
        raise MpcdError(f"{what} failed ({_STATUS.get(rc, rc)}): {msg}", rc)


def param_spec(desc):
    """[(name, shape)] in blob order, straight from the library (single source of truth)."""
    L = lib()
    n_t, n_f = ctypes.c_int32(), ctypes.c_int64()
    check(L.mpcd_net_param_count(ctypes.byref(desc), ctypes.byref(n_t), ctypes.byref(n_f)), "mpcd_net_param_count")
    out = []
    buf = ctypes.create_string_buffer(256)
    nd = ctypes.c_int32()
    shp = (ctypes.c_int64 * 4)()
    for i in range(n_t.value):
        check(L.mpcd_net_param_info(ctypes.byref(desc), i, buf, 256, ctypes.byref(nd), shp), "mpcd_net_param_info")
        out.append((buf.value.decode(), tuple(shp[k] for k in range(nd.value))))
    return out
