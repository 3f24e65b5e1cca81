"""Scan gfx950 assembly for a transcendental VALU result (v_exp_f32 / v_rcp_f32 / v_log_f32 / v_sqrt_f32 /
v_rsq_f32 / v_sin_f32 / v_cos_f32) read by a packed-math VALU op (v_pk_*) within `window` instructions with no
s_nop between them. Usage: python tools/isa/trans_hazard.py file.s [window]  (or a code object via
llvm-objdump -d output). Prints per-kernel counts and the first few sites."""
import re
import sys

TRANS = re.compile(r"^\s*(v_(exp|rcp|log|sqrt|rsq|sin|cos)_f32)\S*\s+v(\d+)")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(operands):
    out = set()
    for m in VREG.finditer(operands):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def scan(lines, window=4):
    sites, kernel = [], None
    insts = []
    for ln in lines:
        s = ln.split(";")[0].rstrip()
        if re.match(r"^[A-Za-z_.$][\w.$]*:\s*$", s) and not s.startswith("."):
            if not s.startswith(".L"):
                kernel = s[:-1]
            continue
        t = s.strip()
        if not t or t.startswith("."):
            continue
        insts.append((kernel, t))
    for i, (k, t) in enumerate(insts):
        m = TRANS.match(t)
        if not m:
            continue
        dst = int(m.group(3))
        for j in range(i + 1, min(i + 1 + window, len(insts))):
            kj, u = insts[j]
            op = u.split()[0]
            if op.startswith("s_nop"):
                break
            parts = u.split(None, 1)
            if len(parts) < 2:
                continue
            ops = [x.strip() for x in parts[1].split(",")]
            srcs = regs(",".join(ops[1:])) if op.startswith("v_") else set()
            if op.startswith("v_pk_") and dst in srcs:
                sites.append((k, i, t, u, j - i))
                break
            if dst in regs(ops[0]) if ops else False:
                break
    return sites


if __name__ == "__main__":
    path = sys.argv[1]
    window = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    with open(path) as f:
        sites = scan(f.readlines(), window)
    per = {}
    for k, *_ in sites:
        per[k] = per.get(k, 0) + 1
    print(f"{len(sites)} trans -> v_pk_* reads within {window} instructions, {len(per)} kernels")
    for k, i, t, u, dist in sites[:8]:
        print(f"  {k[:70]} +{dist}: {t}  ->  {u}")
