"""Summarise the sqpmc passes of tools/gpu.sh (SQ counters of the MLP sampler kernel) into one JSON.

    python tools/sq_summary.py <out.json> <kernel substring> <pass dir> [<pass dir> ...]

Per counter: the mean per launch over the warm launches (all but the first) of the kernels whose name contains the
substring. Derived, per SIMD of the busy CUs: issue shares from SQ_ACTIVE_INST_ANY / SQ_WAIT_INST_ANY / SQ_WAIT_ANY
over SQ_WAVE_CYCLES (all in quad-cycles), the matrix pipe's busy share (SQ_VALU_MFMA_BUSY_CYCLES, cycles) over the
kernel's shader cycles (GRBM_GUI_ACTIVE / 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back')."""
import csv
import json
import sys


def main(out, kern, *dirs):
    vals, name = {}, None
    for d in dirs:
        rows = [r for r in csv.DictReader(open(d + "/run_counter_collection.csv")) if kern in r["Kernel_Name"]]
        by = {}
        for r in rows:
            by.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            by[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            name = r["Kernel_Name"]
        for c, per in by.items():
            v = [per[k] for k in sorted(per, key=int)]
            warm = v[1:] or v
            vals[c] = sum(warm) / len(warm)
    res = {"kernel": name, "per_launch": vals}
    d = {}
    if "SQ_WAVE_CYCLES" in vals:
        wc = vals["SQ_WAVE_CYCLES"]
        for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS"):
            if k in vals:
                d[k + "_share_of_wave_cycles"] = vals[k] / wc
    if "GRBM_GUI_ACTIVE" in vals and "SQ_WAVES" in vals:
        d["shader_cycles_per_launch"] = vals["GRBM_GUI_ACTIVE"] / 8
    if "SQ_INSTS_MFMA" in vals and "SQ_WAVES" in vals:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD"):
            if k in vals:
                d[k + "_per_wave"] = vals[k] / vals["SQ_WAVES"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "SQ_WAVES" in vals and "shader_cycles_per_launch" in d:
        # one wave per SIMD (mlp_rw): busy cycles per wave over the launch's shader cycles
        d["mfma_busy_share_per_simd"] = vals["SQ_VALU_MFMA_BUSY_CYCLES"] / vals["SQ_WAVES"] / d["shader_cycles_per_launch"]
    res["derived"] = d
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
