"""Headline benchmark: candidate trajectories denoised + cost-ranked per second.

BASELINE.json metric "candidate trajectories/sec (100 denoise steps, H=32)", workload = configs[1]:
2D double integrator, 4096 candidates per GPU, H=32, 100 CFG-DDPM steps, MLP noise-net
(build-defined CFG MLP), fp32. One step = one mpc_step: Philox x_T + 100 CFG
denoise steps (200 net evaluations) + unnormalise + fp64 rollout/cost + argmin (+ RCCL cost
all-gather and winner broadcast for N > 1) + the applied action copied to the host.
Weak scaling: every rank adds 4096 candidates.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CFG = dict(workload="cfg2: 2D double integrator, MLP noise-net, CFG-DDPM", system="double_int2d", d=2, H=32, C=4,
           N=100, B=4096, w=0.01, schedule="exponential")
MAC_FWD = 119552          # MLP MACs per forward at H*d = 64 (incl. time MLP + cond projections)
MAC_ROW = 95232           # MACs the kernel executes per row and step: the 14 per-row Linears (time MLP and
                          # cond projections run once per step / per context in the prologues)
PEAK_FP32 = 157.3e12      # MI355X dense fp32 MFMA / vector peak, FLOP/s (MI355X_MICROARCH.md)
PEAK_BF16 = 2516.6e12     # MI355X dense bf16 MFMA peak: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz
PMC_FILES = {"f32": os.path.join(ROOT, "profiles", "r1_pmc_mlp_sampler.json"),
             "f32x3": os.path.join(ROOT, "profiles", "r1_pmc_mlp_x3.json")}


def _rank_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def cpu_baseline(budget_s=12.0, b_cpu=256):
    """The oracle (torch-CPU restatement of the reference path, 'port') on this host's cores:
    normalise -> CFG-DDPM (2 forwards/step) -> unnormalise -> fp64 C rollout/cost -> argmin."""
    from oracle import nets, normalizer, sampler, schedule
    from oracle import systems as osys
    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16)
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    net = nets.ConditionedMLPNet(state_dim=CFG["d"], horizon=CFG["H"], context_dim=CFG["C"]).eval()
    bufs = schedule.buffers(CFG["schedule"], CFG["N"])
    rng = np.random.default_rng(1)
    one = torch.ones(CFG["C"], dtype=torch.float32)
    done, t0 = 0, time.perf_counter()
    while True:
        x0 = rng.uniform(-1, 1, CFG["C"])
        ctx = normalizer.normalize(torch.from_numpy(x0)[None], -one, one).float()
        x = sampler.ddpm_cfg(net, bufs, ctx.expand(b_cpu, CFG["C"]), CFG["w"], b_cpu, CFG["H"])
        u = normalizer.unnormalize(x, -torch.ones(CFG["d"]), torch.ones(CFG["d"]))
        cost = osys.rollout_cost(CFG["system"], x0, u.double().numpy())
        osys.argmin(cost)
        done += b_cpu
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": done / el, "unit": "candidate trajectories/s", "cores": threads, "kind": "port",
            "sample": f"{done // b_cpu} mpc_steps x {b_cpu} candidates (N=100, H=32) in {el:.1f} s; "
                      "linear in B"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--dtype", default="f32x3", choices=["f32", "f32x3"],
                    help="MLP GEMM numerics: exact fp32 MFMA, or fp32-accurate split-bf16 MFMA")
    args = ap.parse_args()

    rank, world, local = _rank_env()
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, systems
    from mpc_via_diffusion_model_amd import distributed as D
    from oracle import nets  # random-init weights of the net's architecture (seed 0), test infra only

    torch.manual_seed(0)
    net = nets.ConditionedMLPNet(state_dim=CFG["d"], horizon=CFG["H"], context_dim=CFG["C"])
    spec = NetSpec("mlp", state_dim=CFG["d"], horizon=CFG["H"], context_dim=CFG["C"], dtype=args.dtype)
    plan = DiffusionMPC(spec, net.state_dict(), variance_schedule=CFG["schedule"], n_diffusion_steps=CFG["N"])
    del net
    system = systems.get(CFG["system"])
    rng = np.random.default_rng(1)
    x0s = rng.uniform(-1, 1, (args.warmup + args.steps, system.n_x))

    # the per-step exchange runs inside libmpcd.so (RCCL communicator of the planner's context)
    comm = D.NativeComm(plan) if world > 1 else None

    def step(i):  # one mpcd_mpc_step call: sample, clip flag, rollout/cost, select, one D2H copy
        return plan.mpc_step(x0s[i], system, CFG["B"], w=CFG["w"], seed=2 + i, comm=comm)

    for i in range(args.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        r = step(args.warmup + i)
        kernel_ms.append(plan.last_sample_ms())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed, float(np.mean(kernel_ms))], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kms = float(t[0]), float(t[1])
    else:
        kms = float(np.mean(kernel_ms))

    if rank == 0:
        total = CFG["B"] * world * args.steps
        flops_launch = CFG["B"] * CFG["N"] * 2 * 2 * MAC_FWD   # survey's algorithmic count (fp32 FLOPs)
        achieved = flops_launch / (kms * 1e-3)
        if args.dtype == "f32x3":
            # executed matrix-core work: six bf16 partial products per fp32 MAC of the per-row Linears
            mfma_flops = CFG["B"] * 2 * CFG["N"] * MAC_ROW * 2 * 6
            roof = {"bound": "mfma", "achieved": mfma_flops / (kms * 1e-3) / 1e12, "peak": PEAK_BF16 / 1e12,
                    "unit": "TFLOP/s", "frac": mfma_flops / (kms * 1e-3) / PEAK_BF16,
                    "peak_note": "bf16 dense MFMA peak; the kernel computes fp32-accurate GEMMs as 3-way bf16 splits",
                    "fp32_equiv": {"achieved": achieved / 1e12, "peak": PEAK_FP32 / 1e12,
                                   "frac": achieved / PEAK_FP32, "flop_per_launch": flops_launch},
                    "kernel": "mlp_x3_kernel<64,DDPM_CFG,ctx>", "flop_per_launch": mfma_flops}
        else:
            roof = {"bound": "mfma", "achieved": achieved / 1e12, "peak": PEAK_FP32 / 1e12, "unit": "TFLOP/s",
                    "frac": achieved / PEAK_FP32, "kernel": "mlp_sample_kernel<64,DDPM_CFG,ctx>",
                    "flop_per_launch": flops_launch}
        traffic = None
        if os.path.exists(PMC_FILES[args.dtype]):
            with open(PMC_FILES[args.dtype]) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        out = {
            "metric": "candidate trajectories/sec (100 denoise steps, H=32)",
            "value": total / elapsed,
            "unit": "candidate trajectories/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (random-init weights seed 0, x0 ~ U[-1,1]^4, Philox noise)",
            "config": {"workload": CFG["workload"], "candidates_per_gpu": CFG["B"], "horizon": CFG["H"],
                       "action_dim": CFG["d"], "context_dim": CFG["C"], "denoise_steps": CFG["N"],
                       "sampler": "CFG-DDPM w=0.01", "schedule": CFG["schedule"], "parallelism": f"dp{world}",
                       "gemm": {"f32": "exact fp32 MFMA (v_mfma_f32_16x16x4_f32)",
                                "f32x3": "fp32-accurate split-bf16 MFMA (3 bf16 terms per operand, 6 partial "
                                         "products, fp32 accumulate)"}[args.dtype]},
            "roofline": dict(roof, traffic=traffic, kernel_ms=kms),
            "best_cost_last_step": r.best_cost,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_budget)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
