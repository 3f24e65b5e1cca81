"""LDS bank-conflict model of the fused U-Net's B-fragment reads (ds_read_b128: 4 lane groups of 16,
bank = dword mod 64, MI355X_MICROARCH.md §LDS) for one (R, H) program: per op, LDS-array cycles per
wave-instruction averaged over the wave's column tiles and K chunks (4 = conflict-free).
    python tools/lds_banks.py R H [cs_rule]"""
import sys

R, H = int(sys.argv[1]), int(sys.argv[2])
RULE = sys.argv[3] if len(sys.argv) > 3 else "32mod64"
GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def cs_of(C):
    cs = (2 * C + 15) // 16 * 16
    if RULE == "32mod64":
        while cs % 64 != 32:
            cs += 16
    elif RULE == "odd16":
        while (cs // 16) % 2 == 0:
            cs += 16
    return cs


def b128_cycles(addr):  # addr[lane] byte address of a 16-byte read
    worst = 0
    for g in GROUPS:
        banks = {}
        for l in g:
            for k in range(4):
                dw = addr[l] // 4 + k
                banks.setdefault(dw % 64, set()).add(dw)
        worst += max(len(v) for v in banks.values())
    return worst


def op_cycles(kind, cinp, L_in, L_out, cs, rowB, lcol):
    kc_n = (({"same5": 5, "down3": 3, "up4": 2, "pw1": 1}[kind]) * cinp + 31) // 32
    ntiles = (R * (2 * L_in if kind == "up4" else L_out)) // 16
    tot = n = 0
    for t in range(ntiles):
        for kc in range(kc_n):
            addr = []
            for lane in range(64):
                col, q = lane & 15, lane >> 4
                c = t * 16 + col
                if kind == "up4":
                    tp = R * L_in // 16
                    par = 1 if t >= tp else 0
                    c -= par * tp * 16
                    cr, m = c // L_in, c % L_in
                    pos0 = m + 1 if par else m
                else:
                    cr, co = c // L_out, c % L_out
                    pos0 = {"same5": co - 2, "down3": 2 * co - 1, "pw1": co}[kind]
                if cinp == 8:
                    tap, ci = 4 * kc + q, 0
                else:
                    cpt = cinp // 32
                    tap, ci = kc // cpt, (kc % cpt) * 32 + 8 * q
                if kind == "up4":
                    tap = -tap
                addr.append(4096 + cr * rowB + (pos0 + tap) * cs + 2 * ci)
            tot += b128_cycles(addr)
            n += 1
    return tot / n


H1, H2 = H // 2, H // 4
ops = [  # (name, kind, cinp, L_in, view channels total of the input)
    ("x same5", "same5", 8, H, 8), ("l0 same5", "same5", 32, H, 32), ("down0", "down3", 32, H, 32),
    ("l1 same5 c32", "same5", 32, H1, 32), ("l1 same5", "same5", 64, H1, 64), ("down1", "down3", 64, H1, 64),
    ("l2 same5 c64", "same5", 64, H2, 64), ("l2 same5", "same5", 128, H2, 128), ("mid (cat2hi)", "same5", 128, H2, 256),
    ("ups0 same5 cat", "same5", 256, H2, 256), ("ups0 same5", "same5", 64, H2, 64), ("up0", "up4", 64, H2, 64),
    ("ups1 same5 cat", "same5", 128, H1, 128), ("ups1 same5", "same5", 32, H1, 32), ("up1", "up4", 32, H1, 32),
    ("final", "same5", 32, H, 32)]
for name, kind, cinp, L_in, ctot in ops:
    cs = cs_of(ctot) if ctot > 8 else cs_of(8)
    L_out = L_in // 2 if kind == "down3" else 2 * L_in if kind == "up4" else L_in
    rowB = (L_in + (7 if ctot == 8 else 2)) * cs
    print(f"{name:16s} cs={cs:4d} rowB={rowB:6d} L_out={L_out:3d}: {op_cycles(kind, cinp, L_in, L_out, cs, rowB, 0):.2f} cycles/read (4 = free)")
