"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/gpu_full.sh) into profiles/<name>.json.

    python tools/pmc_summary.py <fetch_dir> <write_dir> <kernel label> <out.json> [<kernel substring> [<grid size>]]

Per-launch HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (MI355X_MICROARCH.md: on gfx950 FETCH_SIZE tallies
half the bytes of 16-B/lane streaming reads; WRITE_SIZE is exact for 16-B stores). The first launch of the
process is cold (weights not yet in the Infinity Cache / L2) and is reported separately."""
import csv
import json
import os
import sys


def vals(d, counter, only=None, grid=None):
    """per-launch values of one counter; only: substring the kernel name must contain (e.g. "32, 8>"); grid: the
    launches' grid size (the bench's own launches, not its shard-probe launches of the same kernel)"""
    rows = [r for r in csv.DictReader(open(d + "/run_counter_collection.csv"))
            if (not only or only in r["Kernel_Name"]) and (not grid or int(r["Grid_Size"]) == int(grid))]
    v = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == counter]
    return v, rows[0]["Kernel_Name"]


def main(fetch_dir, write_dir, label, out, only=None, grid=None):
    f, kname = vals(fetch_dir, "FETCH_SIZE", only, grid)
    w, _ = vals(write_dir, "WRITE_SIZE", only, grid)
    warm_f = sum(f[1:]) / len(f[1:])
    warm_w = sum(w[1:]) / len(w[1:])
    res = {"kernel": kname, "label": label,
           "command": "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE -- "
                      "python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --dtype <dt> (one pass per counter)",
           "FETCH_SIZE_kb_per_launch": f, "WRITE_SIZE_kb_per_launch": w,
           "hbm_bytes_per_launch": int((2 * warm_f + warm_w) * 1024),
           "hbm_bytes_cold_first_launch": int((2 * f[0] + w[0]) * 1024),
           "hbm_bytes_note": "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 averaged over the warm launches (2..n)"}
    if only:
        res["kernel_filter"] = only
    if grid:
        res["grid_size_filter"] = int(grid)
    # sha256 of the library the passes ran on (tools/gpu.sh pmc writes it beside the pass directories)
    sha = os.path.join(os.path.dirname(os.path.abspath(fetch_dir)),
                       os.path.basename(fetch_dir.rstrip("/")).replace("_FETCH_SIZE", "") + "_lib.sha256")
    if os.path.exists(sha):
        res["lib_sha256"] = open(sha).read().split()[0]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:5], *sys.argv[5:7])
