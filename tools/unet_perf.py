"""Quick U-Net throughput probe: one sample_trajectories call at a BASELINE shape (per-GPU shard)."""
import sys, os, time, argparse
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, force_unet_path
from oracle import nets
ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=16384)
ap.add_argument("--H", type=int, default=32)
ap.add_argument("--d", type=int, default=1)
ap.add_argument("--C", type=int, default=2)
ap.add_argument("--N", type=int, default=100)
ap.add_argument("--steps", type=int, default=10, help="DDIM sampling steps (network evaluations)")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--schedule", default="exponential")
ap.add_argument("--dtype", default="f32x3", choices=["f32", "f32x3", "f16", "f16x2"])
ap.add_argument("--fuse", default="", help="MPCD_UNET_FUSE (0 never, 1 always, empty: measured)")
ap.add_argument("--sampler", default="ddim_cfg", choices=["ddim_cfg", "ddpm_cfg"],
                help="ddpm_cfg runs all N steps (--steps ignored); an f16x2 net runs its two-term program only there")
ap.add_argument("--path", default="auto", choices=["auto", "layered", "fused"], help="mpcd_unet_force_path")
a = ap.parse_args()
if a.fuse:
    os.environ["MPCD_UNET_FUSE"] = a.fuse
force_unet_path(a.path)
torch.manual_seed(0)
net = nets.ConditionedTemporalUnet(state_dim=a.d, context_dim=a.C)
plan = DiffusionMPC(NetSpec("unet", a.d, a.H, a.C, dtype=a.dtype), net.state_dict(), variance_schedule=a.schedule, n_diffusion_steps=a.N)
ctx = torch.rand(1, a.C) * 2 - 1
warm = {"ddim_steps": 2} if a.sampler == "ddim_cfg" else {}
plan.sample_trajectories(ctx, a.B, a.H, sample_fn=a.sampler, **warm)
torch.cuda.synchronize()
for _ in range(a.reps):
    t0 = time.perf_counter()
    kw = {"ddim_steps": a.steps} if a.sampler == "ddim_cfg" else {}
    x = plan.sample_trajectories(ctx, a.B, a.H, sample_fn=a.sampler, **kw)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    evals = a.steps + 1 if a.sampler == "ddim_cfg" else a.N
    mac = {32: 9122560, 64: 18209152}.get(a.H, 0) + 896 * (a.C - 5) + 224 * a.H * (a.d - 1)
    fl = a.B * evals * 2 * 2 * mac
    print(f"{a.dtype} path={a.path} fuse={a.fuse or 'auto'} B={a.B} H={a.H}: {el*1e3:.1f} ms for {evals} CFG net evals -> {el/evals*1e3:.2f} ms/eval, "
          f"{fl/el/1e12:.1f} TFLOP/s, {a.B/el*evals/101:.0f} cand/s at 101 evals")
