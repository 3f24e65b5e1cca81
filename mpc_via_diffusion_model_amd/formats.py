"""On-disk formats of the reference around the hot path, host-side only.

* Trained models: `trained_models/<name>/<step>/args.yaml` + `checkpoints/{ema_,}model_current_state_dict.pth`
  (the GaussianDiffusionModel state_dict: "model.<param>" + the 12 schedule buffers). Loaded weights-only
  (`torch.load(..., weights_only=True)`); the net architecture is read from args.yaml
  (`unet_dim_mults_option`, `unet_input_dim`, `n_diffusion_steps`, `variance_schedule`) and from the tensor
  shapes (state_dim, context_dim); the horizon is a property of the (missing) training data, so it is an
  argument (defaults per dataset_subdir below).
* Training tensors (nmpc_multi_process_collect_data.py:323-331): u `[N, H, 1]`, x0 `[N, C]`, J `[N]` as plain
  tensors in `.pt` files.
* Inference dumps (Diffusion_MPC_Inference.py:407-437): `u_diffusion.npy` `[1, T]`, `u_horizon_diffusion.npy`
  `[T, H]`, `x_diffusion_horizon.npy` `[T, H+1, n_x]`, values rounded to 4 decimals as the reference does.
"""
import os

import numpy as np
import torch
import yaml

# temporal_unet.py:14-17
UNET_DIM_MULTS = {0: (1, 2, 4), 1: (1, 2, 4, 8)}
# horizons of the reference datasets (n_support_points comes from the training tensors, not args.yaml)
DATASET_HORIZON = {"CartPole-NMPC": 32, "CartPole-LMPC": 32, "Panda": 128}
TIME_EMB_DIM = 32


def read_args(model_dir):
    """args.yaml of a trained model directory (safe YAML load, plain data only)."""
    with open(os.path.join(model_dir, "args.yaml")) as f:
        return yaml.safe_load(f)


def checkpoint_path(model_dir, use_ema=None, args=None):
    args = args if args is not None else read_args(model_dir)
    ema = args.get("use_ema", True) if use_ema is None else use_ema
    name = "ema_model_current_state_dict.pth" if ema else "model_current_state_dict.pth"
    return os.path.join(model_dir, "checkpoints", name)


def load_state_dict(path):
    """Weights-only load of a state_dict file (no code executed from the file)."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(sd, dict) or not all(isinstance(v, torch.Tensor) for v in sd.values()):
        raise ValueError(f"{path} is not a plain state_dict of tensors")
    return sd


def infer_spec(state_dict, args, horizon=None, dtype="f32"):
    """NetSpec of a reference checkpoint: ConditionedTemporalUnet (4-arg, CFG-masked) or the build's MLP,
    from the tensor shapes and args.yaml."""
    from .planner import NetSpec

    p = {k[6:] if k.startswith("model.") else k: v for k, v in state_dict.items()}
    if "downs.0.0.blocks.0.block.0.weight" in p:  # ConditionedTemporalUnet / TemporalUnet
        w0 = p["downs.0.0.blocks.0.block.0.weight"]
        base, state_dim = int(w0.shape[0]), int(w0.shape[1])
        n_levels = len({k.split(".")[1] for k in p if k.startswith("downs.")})
        mults = tuple(int(p[f"downs.{i}.0.blocks.0.block.0.weight"].shape[0]) // base for i in range(n_levels))
        opt = args.get("unet_dim_mults_option")
        if opt is not None and UNET_DIM_MULTS.get(int(opt)) != mults:
            raise ValueError(f"args.yaml unet_dim_mults_option {opt} disagrees with the tensors ({mults})")
        cond = p.get("downs.0.0.cond_mlp.1.weight")
        context_dim = int(cond.shape[1]) - TIME_EMB_DIM if cond is not None else 0
        kind = "unet"
    elif "downs.0.0.blocks.0._network.0.weight" in p:  # the build's CFG MLP
        w0 = p["downs.0.0.blocks.0._network.0.weight"]
        base, d0 = int(w0.shape[0]), int(w0.shape[1])
        cond = p["downs.0.0.cond_mlp.1.weight"]
        context_dim = int(cond.shape[1]) - TIME_EMB_DIM
        mults = (1, 2, 4)
        if horizon is None:
            raise ValueError("MLP checkpoints need the horizon (input width is H*d)")
        if d0 % horizon:
            raise ValueError(f"input width {d0} is not a multiple of horizon {horizon}")
        state_dim = d0 // horizon
        kind = "mlp"
    else:
        raise ValueError("unrecognised checkpoint layout")
    if horizon is None:
        horizon = DATASET_HORIZON.get(str(args.get("dataset_subdir", "")).split("/")[0])
        if horizon is None:
            raise ValueError(f"horizon unknown for dataset {args.get('dataset_subdir')!r}: pass horizon=")
    return NetSpec(kind, state_dim=state_dim, horizon=int(horizon), context_dim=context_dim, base_dim=base,
                   dim_mults=mults, cfg=True, dtype=dtype)


def load_trained(model_dir, horizon=None, use_ema=None, context_limits=None, action_limits=None, dtype="f32",
                 device=None):
    """DiffusionMPC of a reference trained-model directory (e.g. trained_models/cart_pole_84000_test1/final).
    The checkpoint's own schedule buffers are used (a recomputation differs by 1 ulp in places). Normaliser
    limits come from the user (the training data they were computed from is not shipped)."""
    from .planner import DiffusionMPC

    args = read_args(model_dir)
    if not args.get("predict_epsilon", True):
        raise ValueError("x0-predicting checkpoints are not on the hot path")
    sd = load_state_dict(checkpoint_path(model_dir, use_ema, args))
    spec = infer_spec(sd, args, horizon, dtype)
    return DiffusionMPC.from_state_dict(sd, spec, variance_schedule=args.get("variance_schedule", "exponential"),
                                        n_diffusion_steps=int(args.get("n_diffusion_steps", 100)),
                                        context_limits=context_limits, action_limits=action_limits, device=device)


# ---------------------------------------------------------------- training tensors
def save_training_tensors(folder, u, x0, cost=None, prefix=""):
    """u [N, H, d], x0 [N, C] (and J [N]) as the data-collection scripts write them (torch.save of plain tensors)."""
    os.makedirs(folder, exist_ok=True)
    u, x0 = torch.as_tensor(u), torch.as_tensor(x0)
    if u.dim() != 3 or x0.dim() != 2 or u.shape[0] != x0.shape[0]:
        raise ValueError("u must be [N, H, d] and x0 [N, C] with the same N")
    n, h, c = u.shape[0], u.shape[1], x0.shape[1]
    paths = {"u": os.path.join(folder, f"{prefix}u_tensor_{n}-{h}-{u.shape[2]}.pt"),
             "x0": os.path.join(folder, f"{prefix}x0_tensor_{n}-{c}.pt")}
    torch.save(u.contiguous(), paths["u"])
    torch.save(x0.contiguous(), paths["x0"])
    if cost is not None:
        paths["J"] = os.path.join(folder, f"{prefix}j_tensor_{n}.pt")
        torch.save(torch.as_tensor(cost).contiguous(), paths["J"])
    return paths


def load_training_tensor(path):
    t = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(t, torch.Tensor):
        raise ValueError(f"{path} does not hold a plain tensor")
    return t


# ---------------------------------------------------------------- inference dumps
def save_inference_results(folder, u_applied, u_horizon=None, x_horizon=None):
    """One closed-loop run in the reference's result layout (Diffusion_MPC_Inference.py:407-437).
    u_applied [T] or [T, d] (d = 1 -> u_diffusion.npy [1, T]); u_horizon [T, H(, d)]; x_horizon
    [T, H+1, n_x]. Values rounded to 4 decimals."""
    os.makedirs(folder, exist_ok=True)
    u = np.asarray(u_applied, dtype=np.float64)
    if u.ndim == 2 and u.shape[1] == 1:
        u = u[:, 0]
    out = {"u_diffusion.npy": np.round(u[None] if u.ndim == 1 else u.T, 4)}
    if u_horizon is not None:
        uh = np.asarray(u_horizon, dtype=np.float64)
        out["u_horizon_diffusion.npy"] = np.round(uh[..., 0] if uh.ndim == 3 and uh.shape[2] == 1 else uh, 4)
    if x_horizon is not None:
        out["x_diffusion_horizon.npy"] = np.round(np.asarray(x_horizon, dtype=np.float64), 4)
    for name, arr in out.items():
        np.save(os.path.join(folder, name), arr)
    return sorted(out)


def load_inference_results(folder):
    return {n[:-4]: np.load(os.path.join(folder, n)) for n in sorted(os.listdir(folder)) if n.endswith(".npy")}
