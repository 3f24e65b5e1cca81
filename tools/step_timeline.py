"""Per-control-step GPU timeline of a bench run from a rocprofv3 --kernel-trace CSV (tools/gpu.sh trace:<w>):
the median duration of every kernel of a step and the idle gaps between them, the step being the span from one
sampler start to the next.

  python tools/step_timeline.py gpurun_out/prof/trace_cfg2 [sampler-name-substring]"""
import csv
import glob
import os
import statistics
import sys


def main():
    root = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "mlp_"
    files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {root}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if key in r[2]]
    # the timed loop: the last 50 steps (bench.py default --steps 50) before the shard probes' first sampler of
    # another grid are indistinguishable here, so take every consecutive sampler pair and keep the spans within
    # 1.5x of the median span
    spans = []
    for a, b in zip(starts, starts[1:]):
        spans.append((rows[b][0] - rows[a][0], a, b))
    med = statistics.median(s for s, _, _ in spans)
    keep = [(a, b) for s, a, b in spans if s <= 1.5 * med]
    segs = {}
    for a, b in keep:
        prev_end = rows[a][0]
        for i in range(a, b):
            s, e, n = rows[i]
            short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            segs.setdefault(f"gap before {short}", []).append((s - prev_end) / 1e3 if i > a else 0.0)
            segs.setdefault(f"kernel {short}", []).append((e - s) / 1e3)
            prev_end = e
        segs.setdefault("gap to the next sampler start (host turnaround)", []).append((rows[b][0] - prev_end) / 1e3)
        segs.setdefault("step (sampler start to next sampler start)", []).append((rows[b][0] - rows[a][0]) / 1e3)
    print(f"{len(keep)} steps of {len(spans)} sampler pairs; medians in us")
    for k, v in segs.items():
        if k.startswith("gap before") and max(v) == 0.0:
            continue
        print(f"  {statistics.median(v):10.2f}  {k}")


if __name__ == "__main__":
    main()
