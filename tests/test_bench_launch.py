"""bench.py's rank launcher (the driver runs `bench.py --gpus N` for N = 1, 2, 4, 8).

CPU: `--gpus N` outside torchrun refuses to time fewer GPUs than asked for, and under a launcher --gpus must equal
WORLD_SIZE. GPU (one card): the bench's own per-rank code - launch_ranks, the barrier-bracketed timed loop, the
max-over-ranks timing, rank 0's JSON line - with two ranks on cuda:0 exchanging over gloo (`--exchange gloo`); the
RCCL exchange of the product path needs a GPU per rank, which the driver's 8-GPU node gives."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=300):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def _visible_gpus():
    import torch
    return torch.cuda.device_count()


def test_more_gpus_than_visible_fails_loudly():
    n = max(2, _visible_gpus() + 1)
    r = _run(["--gpus", str(n), "--no-cpu-baseline"], timeout=180)
    assert r.returncode != 0
    assert f"only {_visible_gpus()} GPU(s) visible" in r.stderr, r.stderr[-2000:]


def test_gpus_must_match_the_launchers_world_size():
    r = _run(["--gpus", "4", "--no-cpu-baseline"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=180)
    assert r.returncode != 0
    assert "--gpus must agree" in r.stderr, r.stderr[-2000:]


def _line(r):
    assert r.returncode == 0, f"bench exited {r.returncode}:\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_two_ranks_on_one_gpu_default_is_strong():
    """The default multi-rank line is SURVEY §8d's strong scaling: cfg2's 4,096 candidates split over the ranks,
    value = 4,096 x steps / time; the weak form (4,096 per rank) is reported beside it."""
    out = _line(_run(["--gpus", "2", "--exchange", "gloo", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]))
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["config"]["candidates_total"] == 4096 and out["config"]["candidates_per_gpu"] == 2048
    assert out["config"]["parallelism"] == "dp2" and "gloo" in out["config"]["exchange"]
    assert out["value"] > 0 and out["steps"] == 3 and out["cpu_baseline"] is None
    assert out["dtype"] == "f32" and out["numerics"] == "f32x3"
    wk = out["weak_scaling"]
    assert wk["candidates_total"] == 8192 and wk["candidates_per_gpu"] == 4096 and wk["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_two_ranks_on_one_gpu_weak_reports_the_strong_split():
    out = _line(_run(["--gpus", "2", "--exchange", "gloo", "--scaling", "weak", "--steps", "3", "--warmup", "1",
                      "--no-cpu-baseline"]))
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert out["config"]["candidates_total"] == 8192 and out["config"]["candidates_per_gpu"] == 4096
    st = out["strong_scaling"]
    assert st["candidates_total"] == 4096 and st["candidates_per_gpu"] == 2048 and st["value"] > 0
