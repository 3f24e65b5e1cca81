"""Summarise tools/fused_pmc.sh passes: per-launch mean of every counter for the kernels matching a filter.
    python tools/fpmc_table.py gpurun_out/fpmc cfg5_fused [name-substring]"""
import collections
import csv
import glob
import sys

d, tag = sys.argv[1], sys.argv[2]
flt = sys.argv[3] if len(sys.argv) > 3 else ""
acc = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/{tag}_p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} n={len(v):4d} mean={sum(v) / len(v):.4g}")
m = {k: sum(v) / len(v) for k, v in acc.items()}
if "SQ_WAVE_CYCLES" in m:
    wc = m["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in m:
            print(f"{k} / WAVE_CYCLES = {m[k] / wc:.3f}")
if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
    print(f"MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 256 CU x 4 SIMD) = "
          f"{m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m:
    print(f"LDS bank conflict cycles / LDS active = {m['SQ_LDS_BANK_CONFLICT'] / max(m['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
