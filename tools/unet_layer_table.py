"""Per-layer time vs MFMA work of one U-Net forward from a rocprofv3 kernel trace (tools/gpu_unet_mx.sh).

    python tools/unet_layer_table.py <run_kernel_trace.csv> [rows=32768] [H=32] [d=1] [planes=3]
"""
import csv
import sys


def layers(H, d, base=32, mults=(1, 2, 4)):
    ch = [base * m for m in mults]
    out, L, prev = [], H, d

    def rtb(ci, co, L):
        out.append(("same5", ci, co, L, L, 5))
        if ci != co:
            out.append(("pw1", ci, co, L, L, 1))
        out.append(("same5", co, co, L, L, 5))
    for i, c in enumerate(ch):
        rtb(prev, c, L)
        rtb(c, c, L)
        if i < len(ch) - 1:
            out.append(("down3", c, c, L, L // 2, 3))
            L //= 2
        prev = c
    rtb(ch[-1], ch[-1], L)
    rtb(ch[-1], ch[-1], L)
    for i in range(1, len(ch)):
        co, ci = ch[-i], ch[-1 - i]
        rtb(2 * co, ci, L)
        rtb(ci, ci, L)
        out.append(("up4", ci, ci, L, 2 * L, 2))
        L *= 2
    out.append(("same5", base, base, L, L, 5))
    out.append(("pw1", base, d, L, L, 1))
    return out


def main(path, rows=32768, H=32, d=1, planes=3):
    rows, H, d, planes = int(rows), int(H), int(d), int(planes)
    tr = [r for r in csv.DictReader(open(path)) if "conv" in r["Kernel_Name"]]
    ls = layers(H, d)
    last = tr[-len(ls):]
    tot_t = tot_f = 0
    print(f"{'layer':28s} {'us':>8s} {'GFLOP':>7s} {'TF/s(fp32-eq)':>13s} {'kernel':s}")
    for (k, ci, co, lin, lout, ks), r in zip(ls, last):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        fl = 2.0 * rows * lout * ci * co * ks
        tot_t += us
        tot_f += fl
        name = r["Kernel_Name"].split("conv_")[1][:22]
        print(f"{k:6s} {ci:4d}->{co:4d} L{lin:3d}->{lout:3d}   {us:8.1f} {fl/1e9:7.2f} {fl/us/1e6:13.1f} {name}")
    print(f"total {tot_t:.0f} us, {tot_f/1e9:.1f} GFLOP, {tot_f/tot_t/1e6:.1f} TF/s fp32-equivalent")


if __name__ == "__main__":
    main(*sys.argv[1:])
