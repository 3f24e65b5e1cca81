"""Wait states between a transcendental VALU result and its first packed-math reader, in gfx950 assembly.

For every v_exp / v_rcp / v_log / v_sqrt / v_rsq / v_sin / v_cos _f32 the scan walks forward to the first
instruction that reads its destination VGPR (or overwrites it) and counts the wait states in between (an
instruction counts 1, `s_nop N` counts N + 1). Reads by a packed-math op (v_pk_*) within `--min` wait states
are the pattern behind csrc/unet_mx.hip's per-element register fence: hipcc's SLP-packed
GroupNorm+Mish epilogue inserted one wait state (the gfx940 trans-use rule) before a v_pk_fma_f32 that reads
a v_rcp_f32 result, and that build gave wrong conv outputs on the GPU while the same code with scalar
consumers (the fence, or -fno-slp-vectorize) is exact.

    python tools/isa/trans_hazard.py file.s [--min N]      (a .s from hipcc -S, or llvm-objdump -d text)
Exit status 1 when any packed reader sits closer than N wait states (default 2)."""
import re
import sys

TRANS = re.compile(r"^(v_(exp|rcp|log|sqrt|rsq|sin|cos)_f32)\S*\s+v(\d+)")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
NOP = re.compile(r"^s_nop\s+(\d+)")


def regs(operands):
    out = set()
    for m in VREG.finditer(operands):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def instructions(lines):
    kernel, out = None, []
    for ln in lines:
        s = ln.split(";")[0].split("//")[0].rstrip()
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", s)  # llvm-objdump -d symbol line
        if m:
            kernel = m.group(1)
            out.append((kernel, None))
            continue
        if re.match(r"^[A-Za-z_.$][\w.$]*:\s*$", s) and not s.startswith("."):
            if not s.startswith(".L"):
                kernel = s[:-1]
            out.append((kernel, None))  # a label: control may join here, stop the walk
            continue
        t = s.strip()
        if t and not t.startswith(".") and not t.endswith(":"):
            out.append((kernel, t))
    return out


def scan(lines, horizon=16):
    """[(kernel, trans inst, reader inst, wait states, packed)] for the first reader of every trans result."""
    insts = instructions(lines)
    sites = []
    for i, (k, t) in enumerate(insts):
        m = TRANS.match(t or "")
        if not m:
            continue
        dst, ws = int(m.group(3)), 0
        for j in range(i + 1, min(i + 1 + horizon, len(insts))):
            _, u = insts[j]
            if u is None or u.startswith("s_cbranch") or u.startswith("s_branch") or u.startswith("s_setpc"):
                break
            n = NOP.match(u)
            if n:
                ws += int(n.group(1)) + 1
                continue
            parts = u.split(None, 1)
            ops = [x.strip() for x in parts[1].split(",")] if len(parts) > 1 else []
            if parts[0].startswith("v_") and ops and dst in regs(",".join(ops[1:])):
                sites.append((k, t, u, ws, parts[0].startswith("v_pk_")))
                break
            if parts[0].startswith("v_") and ops and dst in regs(ops[0]):
                break
            ws += 1
    return sites


def main(argv):
    path = argv[1]
    mn = int(argv[argv.index("--min") + 1]) if "--min" in argv else 2
    with open(path) as f:
        sites = scan(f.readlines())
    packed = [s for s in sites if s[4]]
    hist = {}
    for s in packed:
        hist[s[3]] = hist.get(s[3], 0) + 1
    close = [s for s in packed if s[3] < mn]
    print(f"{len(sites)} trans results read; {len(packed)} first read by v_pk_*; wait states -> count "
          f"{dict(sorted(hist.items()))}; {len(close)} packed reads under {mn} wait states "
          f"in {len({s[0] for s in close})} kernels")
    for k, t, u, ws, _ in close[:6]:
        print(f"  {(k or '?')[:60]} {ws}: {t}  ->  {u}")
    return 1 if close else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
