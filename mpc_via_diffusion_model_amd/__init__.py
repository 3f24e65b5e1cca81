"""MI355X-native diffusion-MPC trajectory generator (hot path of XuehuaOvO/MPC_via_Diffusion_Model).

    from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, systems
    planner = DiffusionMPC.from_state_dict(state_dict, NetSpec("unet", state_dim=1, horizon=32, context_dim=5))
    result = planner.mpc_step(x0, systems.cartpole_lin5(), n_samples=4096)

Compute is in libmpcd.so (hand-written HIP for gfx950, built by ``python -m
mpc_via_diffusion_model_amd.build``); see DESIGN.md and include/mpcd.h.
"""
from . import systems
from .planner import ClosedLoopResult, DiffusionMPC, MPCResult, NetSpec, force_unet_path, force_unet_tiling, philox_noise

__all__ = ["ClosedLoopResult", "DiffusionMPC", "MPCResult", "NetSpec", "force_unet_path", "force_unet_tiling", "philox_noise", "systems"]
