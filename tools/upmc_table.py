"""Per-layer PMC table of the last U-Net forward in tools/gpu_unet_pmc.sh output.

    python tools/upmc_table.py <dtype> [n_layers=35]
"""
import collections
import csv
import sys

dt = sys.argv[1]
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 35
per = collections.defaultdict(dict)
names = {}
for g in "abcde":
    try:
        rows = list(csv.DictReader(open(f"gpurun_out/upmc/{dt}_{g}/run_counter_collection.csv")))
    except FileNotFoundError:
        continue
    ids = sorted(set(int(r["Dispatch_Id"]) for r in rows))[-nl:]
    idx = {d: i for i, d in enumerate(ids)}
    for r in rows:
        d = int(r["Dispatch_Id"])
        if d in idx:
            per[idx[d]][r["Counter_Name"]] = per[idx[d]].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
            names[idx[d]] = r["Kernel_Name"].split("conv_mx_kernel")[1][:14]
cols = ["SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_WAVES",
        "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT",
        "FETCH_SIZE", "WRITE_SIZE"]
print("i  kernel         " + " ".join(f"{c.replace('SQ_', '')[:10]:>10s}" for c in cols))
tot = collections.Counter()
for i in sorted(per):
    print(f"{i:2d} {names[i]:14s} " + " ".join(f"{per[i].get(c, 0):10.3g}" for c in cols))
    for c in cols:
        tot[c] += per[i].get(c, 0)
print("tot               " + " ".join(f"{tot[c]:10.3g}" for c in cols))
