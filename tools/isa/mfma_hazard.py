"""VALU-write -> MFMA-read wait states in gfx950 assembly (csrc/mlp_rw.hip's inline-asm MFMAs).

The hardware needs 2 wait states between a VALU instruction (v_*, v_accvgpr_write included) that writes a
register and an MFMA that reads it as srcA, srcB or srcC. The compiler's hazard pass inserts them for the
builtin MFMAs, but the resident-weight sampler issues some MFMAs as inline asm (AGPR weight operands), which
that pass does not treat as MFMAs. This scan walks back from every v_mfma_* to the previous VALU writes of its
source registers (VGPRs and AGPRs) and reports those closer than 2 wait states (an instruction counts 1,
`s_nop N` counts N + 1; a label or branch ends the walk: control may enter from elsewhere).

    python tools/isa/mfma_hazard.py file.s      (a .s from hipcc -S, or llvm-objdump -d text)
Exit status 1 when any MFMA source is written by a VALU op under 2 wait states before it."""
import re
import sys

REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")
NOP = re.compile(r"^s_nop\s+(\d+)")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.update((m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def instructions(lines):
    kernel, out = None, []
    for ln in lines:
        s = ln.split(";")[0].split("//")[0].rstrip()
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", s)
        if m:
            kernel = m.group(1)
            out.append((kernel, None))
            continue
        if re.match(r"^[A-Za-z_.$][\w.$]*:\s*$", s) and not s.startswith("."):
            if not s.startswith(".L"):
                kernel = s[:-1]
            out.append((kernel, None))
            continue
        t = s.strip()
        if t and not t.startswith(".") and not t.endswith(":"):
            out.append((kernel, t))
    return out


def scan(lines, need=2):
    """[(kernel, mfma inst, writer inst, wait states)] for every MFMA source written by a VALU op < need ago."""
    insts = instructions(lines)
    bad = []
    for i, (k, t) in enumerate(insts):
        if not t or not t.startswith("v_mfma"):
            continue
        parts = t.split(None, 1)
        ops = [x.strip() for x in parts[1].split(",")]
        srcs = regs(",".join(ops[1:4]))
        ws = 0
        for j in range(i - 1, max(-1, i - 8), -1):
            _, u = insts[j]
            if u is None or u.startswith("s_cbranch") or u.startswith("s_branch") or u.startswith("s_setpc"):
                break
            n = NOP.match(u)
            if n:
                ws += int(n.group(1)) + 1
                if ws >= need:
                    break
                continue
            up = u.split(None, 1)
            if up[0].startswith("v_") and not up[0].startswith("v_mfma") and len(up) > 1:
                dst = regs(up[1].split(",")[0])
                if dst & srcs:
                    bad.append((k, t, u, ws))
                    break
            ws += 1
            if ws >= need:
                break
    return bad


def result_reads(lines, kernel_filter=None):
    """[(kernel, mfma inst, first VALU access of its result, wait states, kind)] for every v_mfma_*: the walk
    forward stops at the first VALU op that reads the destination (kind "read") or overwrites it without reading
    it (kind "write": a write-after-write of the accumulator, which in the in-place chains of this library is also
    the write-after-read of the in-flight MFMA's srcC), a label or a branch. A following MFMA that reads the
    result as srcA / srcB is reported as a read; one that takes it as srcC continues the chain (forwarding)."""
    insts = instructions(lines)
    out = []
    for i, (k, t) in enumerate(insts):
        if not t or not t.startswith("v_mfma") or (kernel_filter and kernel_filter not in (k or "")):
            continue
        ops = [x.strip() for x in t.split(None, 1)[1].split(",")]
        dst, ws = regs(ops[0]), 0
        for j in range(i + 1, min(len(insts), i + 64)):
            _, u = insts[j]
            if u is None or u.startswith("s_cbranch") or u.startswith("s_branch") or u.startswith("s_setpc"):
                break
            n = NOP.match(u)
            if n:
                ws += int(n.group(1)) + 1
                continue
            up = u.split(None, 1)
            if len(up) > 1 and up[0].startswith("v_"):
                uops = up[1].split(",")
                if up[0].startswith("v_mfma"):
                    if regs(",".join(uops[1:3])) & dst:  # read as srcA / srcB: not a forwarding case, report
                        out.append((k, t, u, ws, "read"))
                        break
                    if regs(uops[0]) & dst and not regs(",".join(uops[3:4])) & dst:
                        break  # overwritten by another MFMA (the matrix pipe orders its own writes)
                    if regs(",".join(uops[3:4])) & dst:
                        break  # srcC of the next MFMA (forwarding): the chain continues there
                else:
                    if regs(",".join(uops[1:])) & dst:
                        out.append((k, t, u, ws, "read"))
                        break
                    if regs(uops[0]) & dst:
                        out.append((k, t, u, ws, "write"))
                        break
            ws += 1
    return out


def main(argv):
    bad = scan(open(argv[1]).read().splitlines())
    for k, t, u, ws in bad[:20]:
        print(f"{k}: {u!r} -> {t!r}: {ws} wait states")
    print(f"{len(bad)} MFMA sources written by a VALU op under 2 wait states before the MFMA")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
