"""U-Net roofline table from `tools/gpu.sh upmc:<cfg>` output (kernel trace + PMC passes).

    python tools/unet_roofline.py <cfg> <B> <H> <d> <C> <dtype> [out.json]

Takes the LAST noise-net forward of the run - one unet_fused_kernel launch (the whole net + that step's update)
on the fused path, or the period of the conv launch sequence (it repeats once the tiling autotune has cached its
picks) layer by layer - and per launch reports duration, HBM bytes (2 x FETCH_SIZE +
WRITE_SIZE, x1024: on gfx950 FETCH_SIZE tallies half the bytes of 16-B/lane streaming reads,
MI355X_MICROARCH.md §HBM) and MFMA busy; per forward the SURVEY §8d algorithmic FLOPs (2 x MAC x rows),
the executed matrix-core FLOPs (x6 for the split-bf16 net, x3 for the two-term fp16 one), and the fractions of the MFMA and HBM peaks.
"""
import csv
import json
import sys

PEAK_BF16 = 2516.6e12  # dense bf16 / fp16 MFMA, FLOP/s
PEAK_HBM = 8.0e12      # bytes/s
N_SIMD = 256 * 4
N_XCD = 8  # GRBM_GUI_ACTIVE is summed over the 8 XCDs (≈ 8 x the kernel's cycles)


def mac_fwd(H, d, C):
    return {32: 9122560, 64: 18209152}[H] + 896 * (C - 5) + 224 * H * (d - 1)


KERNELS = ("conv_mx_kernel", "unet_fused_kernel")


def is_net(name):
    return any(k in name for k in KERNELS)


def conv_rows(path):
    rows = [r for r in csv.DictReader(open(path)) if is_net(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def period(names):
    for p in range(1, len(names) // 2 + 1):
        if names[-p:] == names[-2 * p:-p]:
            return p
    raise SystemExit("no repeating forward found at the end of the trace")


def short(k):
    for n in KERNELS:
        if n in k:
            return n + k.split(n)[1].split("(")[0].replace(" ", "")
    return k


def main(cfg, B, H, d, C, dtype, out=None):
    B, H, d, C = int(B), int(H), int(d), int(C)
    base = f"gpurun_out/uroof/{cfg}"
    tr = conv_rows(f"{base}_trace/run_kernel_trace.csv")
    names = [short(r["Kernel_Name"]) for r in tr]
    p = period(names)
    last = tr[-p:]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in last]
    # PMC passes: per dispatch, counters summed over the rows of that dispatch
    ctr = {}
    for i in range(3):
        rows = [r for r in csv.DictReader(open(f"{base}_p{i}/run_counter_collection.csv"))
                if is_net(r["Kernel_Name"])]
        per = {}
        for r in rows:
            per.setdefault(int(r["Dispatch_Id"]), {"name": short(r["Kernel_Name"])})
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = per[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(
                r["Counter_Value"])
        seq = [per[k] for k in sorted(per)]
        pp = period([s["name"] for s in seq])
        assert pp == p, (i, pp, p)
        for j, s in enumerate(seq[-p:]):
            assert s["name"] == names[-p + j]
            ctr.setdefault(j, {}).update({k: v for k, v in s.items() if k != "name"})
    prods = {"f32x3": 6, "f16x2": 3}.get(dtype, 1)  # partial products per fp32 MAC on the matrix cores
    rows_n = 2 * B
    flop_alg = 2.0 * mac_fwd(H, d, C) * rows_n
    flop_exec = flop_alg * prods
    t = sum(dur)
    hbm = [(2 * ctr[j].get("FETCH_SIZE", 0) + ctr[j].get("WRITE_SIZE", 0)) * 1024 for j in range(p)]
    # SQ_VALU_MFMA_BUSY_CYCLES = 16 cycles per 16x16x32 MFMA summed over all SIMDs (checked against SQ_INSTS_MFMA)
    busy = [ctr[j].get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(ctr[j].get("GRBM_GUI_ACTIVE", 1) / N_XCD * N_SIMD, 1)
            for j in range(p)]
    table = []
    for j in range(p):
        # executed matrix-core FLOPs of the launch: SQ_INSTS_MFMA (per wave) x 16x16x32 x 2
        fl = ctr[j].get("SQ_INSTS_MFMA", 0) * 16 * 16 * 32 * 2
        table.append({"i": j, "kernel": names[-p + j], "us": round(dur[j] * 1e6, 1),
                      "mfma_gflop": round(fl / 1e9, 1), "mfma_frac": round(fl / dur[j] / PEAK_BF16, 3),
                      "hbm_MB": round(hbm[j] / 1e6, 1),
                      "GB_s": round(hbm[j] / dur[j] / 1e9, 1), "hbm_frac": round(hbm[j] / dur[j] / PEAK_HBM, 3),
                      "mfma_busy": round(busy[j], 3), "mfma_insts": ctr[j].get("SQ_INSTS_MFMA", 0),
                      # issue: SQ_INSTS_VALU counts the MFMAs too; the other VALU instructions occupy the SIMD's
                      # vector pipe >= 4 cycles each (transcendentals 8), per SIMD-cycle of the launch
                      "valu_insts": ctr[j].get("SQ_INSTS_VALU", 0), "lds_insts": ctr[j].get("SQ_INSTS_LDS", 0),
                      "valu_pipe_share_min": round(4 * (ctr[j].get("SQ_INSTS_VALU", 0) - ctr[j].get("SQ_INSTS_MFMA", 0))
                                                   / max(ctr[j].get("GRBM_GUI_ACTIVE", 1) / N_XCD * N_SIMD, 1), 3)})
    res = {
        "config": cfg, "B": B, "rows": rows_n, "H": H, "d": d, "C": C, "dtype": dtype,
        "source": "rocprofv3 --kernel-trace (durations) and three --pmc passes (FETCH_SIZE | WRITE_SIZE | "
                  "SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_MFMA, GRBM_GUI_ACTIVE, ...) over tools/unet_perf.py; "
                  "the last noise-net forward of the run",
        "launches_per_forward": p,
        "form": "fused (one launch per denoise step: the whole net + the update)" if "unet_fused" in names[-1]
                else "layer by layer (one launch per conv)",
        "forward_ms": round(t * 1e3, 3),
        "algorithmic_flop_per_forward": flop_alg,
        "executed_mfma_flop_per_forward": flop_exec,
        "mfma_tflops_executed": round(flop_exec / t / 1e12, 1),
        "mfma_frac_executed": round(flop_exec / t / PEAK_BF16, 3),
        "fp32_equiv_tflops": round(flop_alg / t / 1e12, 1),
        "hbm_bytes_per_forward": int(sum(hbm)),
        "hbm_TB_s": round(sum(hbm) / t / 1e12, 2),
        "hbm_frac": round(sum(hbm) / t / PEAK_HBM, 3),
        "mfma_busy_time_weighted": round(sum(b * x for b, x in zip(busy, dur)) / t, 3),
        "per_launch": table,
    }
    sha = f"{base}_lib.sha256"  # tools/gpu.sh upmc: the library the passes ran on
    try:
        res["lib_sha256"] = open(sha).read().split()[0]
    except OSError:
        pass
    s = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(s)
    print(json.dumps({k: v for k, v in res.items() if k != "per_launch"}, indent=1))
    print(f"{'i':>3} {'kernel':30s} {'us':>8} {'GFLOP':>8} {'mfma':>6} {'MB':>8} {'GB/s':>8} {'hbm':>6} {'busy':>6}")
    for r in table:
        print(f"{r['i']:3d} {r['kernel']:30s} {r['us']:8.1f} {r['mfma_gflop']:8.1f} {r['mfma_frac']:6.3f} {r['hbm_MB']:8.1f} "
              f"{r['GB_s']:8.1f} {r['hbm_frac']:6.3f} {r['mfma_busy']:6.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:8])
