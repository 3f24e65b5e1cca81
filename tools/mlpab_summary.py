"""Summarise gpurun_out/mlpab_<variant>.log bench lines (tools/gpu.sh mlpab:<variant>): cand/s, ms per control
step, sampler kernel ms, and the strong-scaling shard probes' ms per step.

    python tools/mlpab_summary.py base wf32 ...
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for v in sys.argv[1:]:
    path = os.path.join(ROOT, "gpurun_out", f"mlpab_{v}.log")
    line = None
    if os.path.exists(path):
        line = next((l for l in open(path) if l.startswith("{")), None)
    if line is None:
        print(f"{v:>10}: no bench line")
        continue
    d = json.loads(line)
    shards = [round(s["ms_per_step"], 3) for s in d.get("strong_shard_probe", {}).get("shards", [])]
    print(f"{v:>10}: {d['value']:12.0f} cand/s  {d['ms_per_step']:.4f} ms/step  kernel {d['roofline']['kernel_ms']:.4f} ms"
          f"  shards (B/2, B/4, B/8) {shards}")
