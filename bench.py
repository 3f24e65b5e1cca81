"""Headline benchmark: candidate trajectories denoised + cost-ranked per second.

BASELINE.json metric "candidate trajectories/sec (100 denoise steps, H=32)". The default workload is
configs[1] (cfg2): 2D double integrator, 4096 candidates, H=32, 100 CFG-DDPM steps, MLP noise-net
(build-defined CFG MLP), fp32-accurate GEMMs (`f32x3`: every fp32 operand as three bf16 terms,
six partial products accumulated in fp32, csrc/mlp_rw.hip). `--dtype f16x2` selects the two-term fp16 kernel
(22 significant bits per operand, fp16 range: NOT fp32 arithmetic, and its line says "dtype": "f16x2"). One step
= one mpc_step, i.e. one mpcd_mpc_step call: context upload, Philox x_T + the denoising loop (2 net evaluations
per step) + clip flag + fp64 rollout/cost + argmin + winner row (+ RCCL cost all-gather and winner exchange for
N > 1) + the applied trajectory to the host. Strong scaling: the workload's B candidates are split
over the ranks; a multi-rank run also times the weak form (B per rank) and reports it beside the value as
"weak_scaling".

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg1..cfg5|panda] [--dtype ...]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`--gpus N` without torchrun starts the N rank processes itself (launch_ranks); under torchrun --gpus must
equal WORLD_SIZE. `--exchange gloo` rehearses the multi-rank bench with every rank on cuda:0.

The other BASELINE configs are selectable with --workload (their lines are kept under profiles/):
cfg1 (the reference's CPU-sized case), cfg3 (pendulum, 1D U-Net, CFG-DDIM 100 steps), cfg4 (cart-pole
NMPC dynamics, U-Net, H=64, fused split-bf16 program), cfg5 (12-DoF quadrotor, U-Net fp16 operands, 250 steps:
the config BASELINE names "fp16 hidden").
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

# SURVEY §8d workloads. mac: algorithmic MACs per noise-net forward;
# mac_row: MACs the kernels execute per row and step on the matrix cores (MLP: the 14 per-row Linears -
# the time MLP and cond projections run once per step / per context in the prologues).
WORKLOADS = {
    "cfg1": dict(workload="cfg1: 2D double integrator, MLP noise-net, CFG-DDPM (reference CPU-sized case)",
                 system="double_int2d", net="mlp", d=2, H=16, C=4, N=50, B=64, sampler="ddpm_cfg",
                 ddim_steps=None, schedule="exponential", dtype="f32x3", mac=117504, mac_row=93184),
    "cfg2": dict(workload="cfg2: 2D double integrator, MLP noise-net, CFG-DDPM", system="double_int2d", net="mlp",
                 d=2, H=32, C=4, N=100, B=4096, sampler="ddpm_cfg", ddim_steps=None,
                 schedule="exponential", dtype="f32x3", mac=119552, mac_row=95232),
    "cfg3": dict(workload="cfg3: pendulum swing-up, 1D temporal U-Net, CFG-DDIM (100 sampling steps)",
                 system="pendulum", net="unet", d=1, H=32, C=2, N=100, B=16384, sampler="ddim_cfg",
                 ddim_steps=100, schedule="exponential", dtype="f32x3", mac=9122560 + 896 * (2 - 5), mac_row=None),
    "cfg4": dict(workload="cfg4: cart-pole (nonlinear NMPC dynamics), 1D temporal U-Net, CFG-DDPM, H=64",
                 system="cartpole_nl5", net="unet", d=1, H=64, C=5, N=100, B=65536, sampler="ddpm_cfg",
                 ddim_steps=None, schedule="exponential", dtype="f32x3", mac=18209152, mac_row=None),
    "cfg5": dict(workload="cfg5: 12-DoF quadrotor, 1D temporal U-Net with fp16 GEMM operands, CFG-DDPM 250 steps",
                 system="quadrotor12", net="unet", d=4, H=64, C=12, N=250, B=131072, sampler="ddpm_cfg",
                 ddim_steps=None, schedule="cosine", dtype="f16", mac=18258432, mac_row=None),
}
PEAK_FP32 = 157.3e12      # MI355X dense fp32 MFMA / vector peak, FLOP/s (MI355X_MICROARCH.md)
PEAK_BF16 = 2516.6e12     # MI355X dense bf16 / fp16 MFMA peak: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz
LIB = os.path.join(ROOT, "mpc_via_diffusion_model_amd", "libmpcd.so")
PMC_FILES = {("cfg2", "f32"): os.path.join(ROOT, "profiles", "r1_pmc_mlp_sampler.json"),
             ("cfg2", "f32x3"): os.path.join(ROOT, "profiles", "r6_pmc_cfg2_mlp_rw.json"),
             ("cfg1", "f32x3"): os.path.join(ROOT, "profiles", "r6_pmc_cfg1_mlp_rw.json"),
             ("cfg2", "f16x2"): os.path.join(ROOT, "profiles", "r5_pmc_mlp_h2.json"),
             # U-Net: HBM bytes of one noise-net forward (the fused launch of one denoise step, PMC FETCH_SIZE x2 +
             # WRITE_SIZE, tools/unet_roofline.py) at B
             ("cfg3", "f32x3"): os.path.join(ROOT, "profiles", "r6_unet_roofline_cfg3.json"),
             ("cfg4", "f32x3"): os.path.join(ROOT, "profiles", "r6_unet_roofline_cfg4.json"),
             ("cfg4", "f16x2"): os.path.join(ROOT, "profiles", "r5_unet_roofline_cfg4_h2.json"),
             ("cfg5", "f16"): os.path.join(ROOT, "profiles", "r6_unet_roofline_cfg5.json")}


def lib_sha256(path=None):
    """sha256 of the loaded product library (MPCD_LIB overrides it, as in _native.py): ties a PMC traffic file to
    the build it was measured on"""
    import hashlib
    path = path or os.environ.get("MPCD_LIB") or LIB
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def _rank_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def synthetic_params(spec, seed=0):
    """Random-init weights of the net's architecture without the oracle: PyTorch's default init restated
    per tensor of the library's parameter list (mpcd_net_param_info): Linear / Conv1d / ConvTranspose1d
    weights and biases ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (kaiming_uniform_(a=sqrt(5)); fan_in =
    size(1) * kernel size, as torch computes it), GroupNorm weight 1 and bias 0. Seeded, CPU."""
    from mpc_via_diffusion_model_amd import _native as N
    g = torch.Generator().manual_seed(seed)
    specs = N.param_spec(spec.desc())
    shapes = dict(specs)
    out = {}
    for name, shp in specs:
        if len(shp) >= 2:
            fan_in = shp[1] * int(np.prod(shp[2:], dtype=np.int64))
        else:
            wshape = shapes.get(name[:-len("bias")] + "weight") if name.endswith("bias") else None
            if wshape is None or len(wshape) < 2:  # GroupNorm affine
                out[name] = torch.ones(shp) if name.endswith("weight") else torch.zeros(shp)
                continue
            fan_in = wshape[1] * int(np.prod(wshape[2:], dtype=np.int64))
        b = 1.0 / np.sqrt(fan_in)
        out[name] = (torch.rand(shp, generator=g, dtype=torch.float64) * 2 - 1).mul(b).float()
    return out


def _net(cfg):
    from oracle import nets  # the CPU baseline's torch module (test infrastructure, cpu_baseline leg only)
    torch.manual_seed(0)
    if cfg["net"] == "mlp":
        return nets.ConditionedMLPNet(state_dim=cfg["d"], horizon=cfg["H"], context_dim=cfg["C"]).eval()
    return nets.ConditionedTemporalUnet(state_dim=cfg["d"], context_dim=cfg["C"]).eval()


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_share():
    """CPUs this process may actually use: os.cpu_count() shows the whole machine on a shared GPU box,
    the affinity mask and the cgroup CPU quota show its share."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(cfg, budget_s=12.0):
    """The oracle (torch-CPU restatement of the reference path, 'port') on this host's cores, SURVEY §8d:
    every CPU this process may use (torch.set_num_threads), B_cpu = min(B, 256) candidates per control
    step, full N: normalise -> CFG sampler (2 forwards/step) -> unnormalise -> fp64 C rollout/cost -> argmin.
    At least one control step, then as many as fit the budget."""
    from oracle import normalizer, sampler, schedule
    from oracle import systems as osys
    threads = _cpu_share()
    torch.set_num_threads(threads)
    b_cpu = min(cfg["B"], 256)
    net = _net(cfg)
    bufs = schedule.buffers(cfg["schedule"], cfg["N"])
    rng = np.random.default_rng(1)
    one = torch.ones(cfg["C"], dtype=torch.float32)
    done, t0 = 0, time.perf_counter()
    while True:
        x0 = rng.uniform(-1, 1, cfg["C"])
        ctx = normalizer.normalize(torch.from_numpy(x0)[None], -one, one).float().expand(b_cpu, cfg["C"])
        if cfg["sampler"] == "ddim_cfg":
            x = sampler.ddim_cfg(net, bufs, ctx, 0.01, b_cpu, cfg["H"], sampling_steps=cfg["ddim_steps"])
        else:
            x = sampler.ddpm_cfg(net, bufs, ctx, 0.01, b_cpu, cfg["H"])
        u = normalizer.unnormalize(x, -torch.ones(cfg["d"]), torch.ones(cfg["d"]))
        cost = osys.rollout_cost(cfg["system"], x0, u.double().numpy())
        osys.argmin(cost)
        done += b_cpu
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": done / el, "unit": "candidate trajectories/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{done // b_cpu} mpc_steps x {b_cpu} candidates (N={cfg['N']}, H={cfg['H']}) in {el:.1f} s "
                      f"on {threads} threads ({_cpu_model()}; {os.cpu_count()} CPUs on the host, {threads} in this "
                      f"process's share); per-candidate cost is linear in B, so cand/s at B={cfg['B']} is the same"}


PANDA_CKPT = os.path.join(ROOT, "tests", "golden", "panda_test6_117600_ema.safetensors")
PANDA_REF_S = 0.3615  # BASELINE.md / SURVEY §6: the reference's median Panda control step (unspecified CUDA GPU)


def panda(args):
    """The reference's one published timing: a Panda control step of
    scripts/Panda/panda_inference/inference_diffusion_panda.py:118-120 / 436-450 - normalise the 20-dim state
    (LimitsNormalizer, fp64 -> fp32), run_CFG(context, None, w=0.01, n_samples=1, horizon=128,
    return_chain=True, ddpm_cart_pole_sample_fn, n_diffusion_steps_without_noise=5) with the trained
    panda_test6_117600 EMA net (ConditionedTemporalUnet d=7, C=20, N=25, the checkpoint's schedule buffers),
    timed host-side around the call and a stream synchronisation, as the reference's time.time() pair around
    diffusion_sampling (its TimerCUDA synchronises). States ~ U[-1, 1]^20 with limits [-1, 1] (the training
    data behind the reference's limits is not shipped). Also: the same step at B = 64 candidates (throughput)."""
    from safetensors.torch import load_file

    from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec
    torch.cuda.set_device(0)
    dtype = args.dtype or "f32x3"
    sd = load_file(PANDA_CKPT)
    plan = DiffusionMPC.from_state_dict(sd, NetSpec("unet", state_dim=7, horizon=128, context_dim=20, dtype=dtype))
    rng = np.random.default_rng(1)
    steps = args.steps if args.steps is not None else 200
    warmup = args.warmup if args.warmup is not None else 10

    def control_step(x, B, i):
        ctx = plan.normalize_condition(x)[None]   # dataset.normalize_condition (host, fp64 -> fp32)
        chain = plan.run_CFG(ctx, None, 0.01, n_samples=B, horizon=128, return_chain=True,
                             n_diffusion_steps_without_noise=5, seed=i)
        torch.cuda.synchronize()
        return chain

    out = {"metric": "Panda control-step latency (run_CFG, B=1, H=128, 25 + 5 CFG-DDPM steps, return_chain)",
           "unit": "s", "higher_is_better": False, "n_gpus": 1, "steps": steps, "warmup": warmup,
           "dtype": {"f32": "f32", "f32x3": "f32", "f16x2": "f16x2", "f16": "f16"}[dtype], "numerics": dtype,
           "data": "trained panda_test6_117600 EMA weights "
           "(tests/golden), synthetic states ~ U[-1,1]^20", "vs_baseline": None,
           "reference_published_s": {"median": PANDA_REF_S, "note": "BASELINE.md / SURVEY §6, unspecified CUDA GPU "
                                     "(eager PyTorch); context only, different hardware"}}
    for B in (1, 64):
        xs = rng.uniform(-1, 1, (warmup + steps, 20))
        for i in range(warmup):
            control_step(xs[i], B, i)
        lat, ker = [], []
        for i in range(steps):
            t0 = time.perf_counter()
            chain = control_step(xs[warmup + i], B, warmup + i)
            lat.append(time.perf_counter() - t0)
            ker.append(plan.last_sample_ms())
        assert tuple(chain.shape) == (31, B, 128, 7) and torch.isfinite(chain).all()
        lat = np.array(lat)
        rec = {"p50_s": float(np.median(lat)), "mean_s": float(lat.mean()), "min_s": float(lat.min()),
               "max_s": float(lat.max()), "kernel_ms_mean": float(np.mean(ker)),
               "candidates_per_s": B / float(np.median(lat))}
        if B == 1:
            out.update(value=rec["p50_s"], ms_per_step=1e3 * rec["p50_s"], latency_b1=rec)
        else:
            out["throughput_b64"] = rec
    form = plan.unet_form("ddpm_cfg")
    out["config"] = {"workload": "panda: trained ConditionedTemporalUnet d=7, C=20, H=128, N=25 + 5 noise-free, CFG w=0.01",
                     "unet_form": form, "gemm": dtype}
    out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, exchange, argv):
    """`bench.py --gpus N` (N > 1) outside torchrun: this parent makes no GPU call (torch.cuda.device_count() does
    not initialise the GPU on this image) and runs N fresh child processes of this same command line, one per GPU,
    each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in its environment - the env rendezvous
    torchrun would give them. Rank 0's stdout (the JSON line) is relayed; the other ranks' stdout goes to stderr.
    The first rank that fails takes the others down and the parent exits with its status."""
    import subprocess
    import threading
    if exchange == "rccl":
        visible = torch.cuda.device_count()
        if visible < n:
            raise SystemExit(f"bench.py --gpus {n}: only {visible} GPU(s) visible; refusing to time {n} ranks on "
                             f"fewer GPUs (--exchange gloo runs every rank on cuda:0 as a rehearsal)")
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))
    lines = []
    reader = threading.Thread(target=lambda: lines.extend(procs[0].stdout), daemon=True)
    reader.start()
    failed = None
    while failed is None and any(p.poll() is None for p in procs):
        failed = next((r for r, p in enumerate(procs) if p.poll() not in (None, 0)), None)
        time.sleep(0.2)
    if failed is None:
        failed = next((r for r, p in enumerate(procs) if p.returncode != 0), None)
    if failed is not None:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p in procs:
        p.wait()
    reader.join(timeout=10)
    for ln in lines:
        sys.stdout.write(ln.decode(errors="replace"))
    sys.stdout.flush()
    if failed is not None:
        raise SystemExit(f"bench.py: rank {failed} of {n} exited with status {procs[failed].returncode}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE under torchrun, else 1); N > 1 without torchrun "
                         "starts the N rank processes itself")
    ap.add_argument("--exchange", default="rccl", choices=["rccl", "gloo"],
                    help="rccl: one GPU per rank, the per-step exchange inside libmpcd.so over RCCL (the product); "
                         "gloo: every rank on cuda:0, the exchange through torch.distributed over gloo (a one-GPU "
                         "rehearsal of the multi-rank bench)")
    ap.add_argument("--steps", type=int, default=None, help="timed control steps (default 50; U-Net configs 5)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed control steps (default 20: the shader clock settles over the first dozen launches; U-Net configs 2, the first one runs the tiling autotune)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong (default, SURVEY §8d): the workload's B_total candidates split over the ranks (a "
                         "multi-rank run also times the weak form beside it); weak: every GPU runs B candidates and "
                         "the units all ranks process add up")
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS) + ["panda"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-shard-probe", action="store_true", help="skip the strong-scaling shard probes (kernel traces)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--candidates", type=int, default=None,
                    help="override the workload's B (profiling a shard size; the line then names the changed config)")
    ap.add_argument("--dtype", default=None, choices=["f32", "f32x3", "f16", "f16x2"],
                    help="GEMM numerics: exact fp32 MFMA, fp32-accurate split-bf16 MFMA (default but cfg5), fp16 "
                         "operands (cfg5), two-term fp16 MFMA (22-bit operands, fp16 range: labelled f16x2)")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if (args.gpus or 1) > 1:
            if args.workload == "panda":
                raise SystemExit("--workload panda is a one-GPU latency bench")
            return launch_ranks(args.gpus, args.exchange, sys.argv[1:])
    elif args.gpus is not None and args.gpus != int(env_world):
        raise SystemExit(f"bench.py --gpus {args.gpus} under a launcher with WORLD_SIZE={env_world}: the rank count "
                         "and --gpus must agree")
    if args.workload == "panda":
        return panda(args)
    cfg = dict(WORKLOADS[args.workload])
    if args.candidates:
        cfg.update(B=args.candidates, workload=cfg["workload"] + f" [B overridden: {args.candidates}]")
    dtype = args.dtype or cfg["dtype"]
    unet = cfg["net"] == "unet"
    steps = args.steps if args.steps is not None else (5 if unet else 50)
    warmup = args.warmup if args.warmup is not None else (2 if unet else 20)
    rank, world, local = _rank_env()
    gloo = world > 1 and args.exchange == "gloo"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if gloo:  # rehearsal: every rank on cuda:0, torch.distributed over gloo
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            visible = torch.cuda.device_count()
            if local >= visible:
                raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {visible} GPU(s) visible")
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        if torch.cuda.device_count() < 1:
            raise SystemExit("bench.py: no GPU visible")
        torch.cuda.set_device(0)
    if cfg["B"] % world:
        raise SystemExit(f"{args.workload}: {cfg['B']} candidates do not split over {world} ranks")
    if args.scaling == "strong":
        b_local, scaling = cfg["B"] // world, "strong"
    else:
        b_local, scaling = cfg["B"], "weak"

    from mpc_via_diffusion_model_amd import DiffusionMPC, NetSpec, systems
    from mpc_via_diffusion_model_amd import distributed as D

    spec = NetSpec(cfg["net"], state_dim=cfg["d"], horizon=cfg["H"], context_dim=cfg["C"], dtype=dtype)
    plan = DiffusionMPC(spec, synthetic_params(spec, seed=0), variance_schedule=cfg["schedule"],
                        n_diffusion_steps=cfg["N"])
    system = systems.get(cfg["system"])
    assert system.n_x == cfg["C"] and system.n_u == cfg["d"]
    rng = np.random.default_rng(1)
    x0s = rng.uniform(-1, 1, (warmup + steps, system.n_x))
    n_evals = plan.n_denoise_steps(cfg["sampler"], 0, cfg["ddim_steps"])  # CFG steps (2 forwards each)
    # rccl: the per-step exchange runs inside libmpcd.so (RCCL communicator of the planner's context);
    # gloo rehearsal: the composed step, exchange through torch.distributed (distributed.select)
    comm = D.NativeComm(plan) if world > 1 and not gloo else None

    def step(i, b):  # one mpc_step (rccl / one rank: one mpcd_mpc_step call) of b candidates on this rank
        return plan.mpc_step(x0s[i], system, b, w=0.01, sample_fn=cfg["sampler"], ddim_steps=cfg["ddim_steps"],
                             seed=2 + i, comm=comm)

    def timed(b):
        """warmup + steps control steps of b candidates per rank between barriers; (wall s, mean kernel ms,
        last result), both maxima over ranks"""
        for i in range(warmup):
            step(i, b)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            res = step(warmup + i, b)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # the sampler launches' HIP events of the timed steps, read once afterwards (no host query inside the loop)
        kms = plan.sample_ms_mean(min(steps, 256))
        if world > 1:
            t = torch.tensor([el, kms], dtype=torch.float64, device="cpu" if gloo else "cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t[0]), float(t[1]), res
        return el, kms, res

    elapsed, kms, r = timed(b_local)
    # a multi-rank run also times the other form in the same job: weak beside a strong value (B per rank, the
    # units of all ranks added), strong beside a weak one (the workload's B over the ranks)
    other = None
    if world > 1:
        b_o = cfg["B"] if scaling == "strong" else cfg["B"] // world
        el_o, kms_o, r_o = timed(b_o)
        other = {"candidates_total": b_o * world, "candidates_per_gpu": b_o, "steps": steps,
                 "value": b_o * world * steps / el_o, "ms_per_step": 1e3 * el_o / steps, "kernel_ms": kms_o,
                 "best_cost_last_step": r_o.best_cost}

    # strong scaling: the shard each of P = 2, 4, 8 GPUs gets (B_total / P candidates), measured here on one GPU;
    # (ms_per_step at B_total) / (ms_per_step at B_total / P) is the compute-only P-GPU speedup bound
    shard_probe = []
    if world == 1 and not args.no_shard_probe:
        ms_full = 1e3 * elapsed / steps
        for div in (2, 4, 8):
            if cfg["B"] % div:
                continue
            bs = cfg["B"] // div
            nw, n1 = (1, max(2, steps // 2)) if unet else (5, max(steps, 20))
            for i in range(nw):
                plan.mpc_step(x0s[i % len(x0s)], system, bs, w=0.01, sample_fn=cfg["sampler"],
                              ddim_steps=cfg["ddim_steps"], seed=100 + i)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for i in range(n1):
                plan.mpc_step(x0s[i % len(x0s)], system, bs, w=0.01, sample_fn=cfg["sampler"],
                              ddim_steps=cfg["ddim_steps"], seed=200 + i)
            torch.cuda.synchronize()
            el1 = time.perf_counter() - t1
            shard_probe.append({"gpus": div, "candidates": bs, "steps": n1, "value": bs * n1 / el1,
                                "ms_per_step": 1e3 * el1 / n1, "speedup_bound": ms_full / (1e3 * el1 / n1)})

    if rank == 0:
        total = b_local * world * steps
        flops_launch = b_local * n_evals * 2 * 2 * cfg["mac"]   # survey's algorithmic count (fp32 FLOPs)
        achieved = flops_launch / (kms * 1e-3)
        if not unet:
            form = plan.mlp_form(b_local, cfg["sampler"])
            tmpl = "%d,DDPM_CFG,ctx" % (cfg["H"] * cfg["d"])
            if form["kernel"] == "f32":
                kname = "mlp_sample_kernel<%s>" % tmpl
            elif form["kernel"] == "h2":
                kname = "mlp_h2_kernel<%s,%d>" % (tmpl, form["rows_per_workgroup"])
            elif form["layout"].startswith("rw"):
                kname = "mlp_rw_kernel<%s,%s>" % (tmpl, form["layout"][2:])
            else:
                r_, w_ = form["layout"].split("x")
                kname = "mlp_x3_kernel<%s,%s,%s>" % (tmpl, r_, w_)
            timed_desc = f"{kname}: the whole denoising loop in one persistent launch (HIP events on the call's stream)"
        else:
            form = plan.unet_form(cfg["sampler"])
            if form["fused"]:
                kname = "unet_fused_kernel<%d,%d,%d,%d>" % (form["planes"], form["rows_per_workgroup"], cfg["H"],
                                                            form["waves_per_workgroup"])
                timed_desc = (f"one mpcd_sample call: {n_evals} {kname} launches (per denoise step the whole noise net "
                         "for both CFG branches + the update, activations in LDS) + the x_T / chain-maxima kernels "
                         "(HIP events on the call's stream); the fused launches are >99% of it (profiles/)")
            else:
                kname = "conv_mx_kernel<kind,planes,NN,NC> family" if dtype != "f32" else "conv_kernel family"
                timed_desc = ("one mpcd_sample call: every U-Net conv launch of the loop + the per-step update kernels "
                         "(HIP events on the call's stream); the convs are >99% of it (profiles/)")
        if dtype in ("f32x3", "f16x2"):
            mac_exec = cfg["mac_row"] if cfg["mac_row"] else cfg["mac"]
            # 3 partial products for the two-term fp16 kernels (the MLP's h2 kernel, the fused U-Net's P = 2 program)
            prods = 3 if (dtype == "f16x2" and (form["fused"] if unet else form["kernel"] == "h2")) else 6
            mfma_flops = b_local * 2 * n_evals * mac_exec * 2 * prods   # bf16 / fp16 partial products per fp32 MAC
            roof = {"bound": "mfma", "achieved": mfma_flops / (kms * 1e-3) / 1e12, "peak": PEAK_BF16 / 1e12,
                    "unit": "TFLOP/s", "frac": mfma_flops / (kms * 1e-3) / PEAK_BF16,
                    "peak_note": ("fp16 dense MFMA peak (= bf16); the kernel computes fp32-class GEMMs as two fp16 terms "
                                  "per operand (3 partial products per fp32 MAC)") if prods == 3 else
                                 ("bf16 dense MFMA peak; the kernels compute fp32-accurate GEMMs as 3-way bf16 splits "
                                  "(6 partial products per fp32 MAC)"),
                    # the same executed MACs at the fp32 rate (the survey's algorithmic count, flops_launch, also
                    # counts the per-candidate time / cond MLPs the kernel computes once per step)
                    "fp32_equiv": {"achieved": mfma_flops / prods / (kms * 1e-3) / 1e12, "peak": PEAK_FP32 / 1e12,
                                   "frac": mfma_flops / prods / (kms * 1e-3) / PEAK_FP32,
                                   "flop_per_launch": mfma_flops / prods, "algorithmic_flop_per_launch": flops_launch},
                    "kernel": kname, "flop_per_launch": mfma_flops}
        elif dtype == "f16":
            roof = {"bound": "mfma", "achieved": achieved / 1e12, "peak": PEAK_BF16 / 1e12, "unit": "TFLOP/s",
                    "frac": achieved / PEAK_BF16, "peak_note": "fp16 dense MFMA peak", "kernel": kname,
                    "flop_per_launch": flops_launch}
        else:
            roof = {"bound": "mfma", "achieved": achieved / 1e12, "peak": PEAK_FP32 / 1e12, "unit": "TFLOP/s",
                    "frac": achieved / PEAK_FP32, "kernel": kname, "flop_per_launch": flops_launch}
        # traffic: HBM bytes per launch from a PMC pass of this workload (FETCH_SIZE x 2 + WRITE_SIZE, tools/
        # pmc_summary.py); the file records the sha256 of the library it was measured on, and the line says whether
        # that is the library this run loaded
        traffic, traffic_source = None, None
        pmc = PMC_FILES.get((args.workload, dtype))
        if pmc and os.path.exists(pmc):
            with open(pmc) as f:
                pm = json.load(f)
            if "hbm_bytes_per_forward" in pm:  # one sample call = n_evals forwards; bytes scale with the rows
                traffic = pm["hbm_bytes_per_forward"] * n_evals * b_local / pm["B"]
            elif pm.get("B", b_local) == b_local or "B" not in pm:
                traffic = pm.get("hbm_bytes_per_launch")
            same = pm.get("lib_sha256") is not None and pm.get("lib_sha256") == lib_sha256()
            traffic_source = {"file": os.path.relpath(pmc, ROOT), "same_build": same,
                              "kind": "PMC pass of this workload on the library this run loaded" if same else
                                      "static: PMC pass of this workload on an earlier build (not re-measured)"}
        gemm = {"f32": "exact fp32 MFMA (v_mfma_f32_16x16x4_f32)",
                "f32x3": "fp32-accurate split-bf16 MFMA (3 bf16 terms per operand, 6 partial products, fp32 accumulate)",
                "f16x2": "two-term fp16 MFMA (hi + lo fp16 per operand: 22 significant bits, the fp16 range; weights "
                         "scaled per layer by a power of two; 3 partial products, fp32 accumulate): NOT fp32 "
                         "arithmetic; the MLP's CFG-DDPM kernel / the fused U-Net, the f32x3 kernels otherwise",
                "f16": "fp16 operands, fp32 accumulate (v_mfma_f32_16x16x32_f16)"}[dtype]
        out = {
            "metric": "candidate trajectories/sec (100 denoise steps, H=32)" if args.workload == "cfg2" else
                      f"candidate trajectories/sec ({n_evals} denoise steps, H={cfg['H']})",
            "value": total / elapsed,
            "unit": "candidate trajectories/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": 1e3 * elapsed / steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            # the arithmetic the GEMMs run: f32x3 reproduces fp32 (three bf16 terms per operand, 24 significant bits,
            # fp32 range, fp32 accumulation); f16x2 (22 bits, fp16 range) and f16 say so
            "dtype": {"f32": "f32", "f32x3": "f32", "f16x2": "f16x2", "f16": "f16"}[dtype],
            "numerics": dtype,
            "data": f"synthetic (random-init weights seed 0 by PyTorch's default-init rule, x0 ~ U[-1,1]^{cfg['C']}, "
                    "Philox noise)",
            "config": {"workload": cfg["workload"], "candidates_per_gpu": b_local, "candidates_total": b_local * world,
                       "horizon": cfg["H"], "action_dim": cfg["d"], "context_dim": cfg["C"], "denoise_steps": n_evals,
                       "sampler": f"{'CFG-DDIM' if cfg['sampler'] == 'ddim_cfg' else 'CFG-DDPM'} w=0.01",
                       "schedule": cfg["schedule"], "noise_net": cfg["net"], "parallelism": f"dp{world}",
                       "exchange": ("none" if world == 1 else "torch.distributed gloo, every rank on cuda:0 "
                                    "(rehearsal)" if gloo else "RCCL inside libmpcd.so (cost all-gather + winner "
                                    "all-reduce), one GPU per rank"),
                       "gemm": gemm},
            "roofline": dict(roof, traffic=traffic, traffic_source=traffic_source, kernel_ms=kms, timed=timed_desc),
            "best_cost_last_step": r.best_cost,
        }
        if other is not None:
            if scaling == "strong":
                out["weak_scaling"] = dict(other, note="the same job's weak form: B candidates per rank, the units "
                                                       "of all ranks added, timed like value (max over ranks)")
            else:
                out["strong_scaling"] = dict(other, note="the same job's strong split: the workload's B candidates "
                                                         "over the ranks, timed like value (max over ranks)")
        if shard_probe:
            out["strong_shard_probe"] = {
                "note": "one GPU running the B_total/P-candidate shard each of P GPUs gets under strong scaling "
                        "(before the per-step exchange); speedup_bound = ms_per_step(B_total) / ms_per_step(shard) "
                        "is the compute-only P-GPU bound",
                "shards": shard_probe}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_budget)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
