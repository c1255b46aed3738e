#!/usr/bin/env python3
"""Scan gfx950 assembly for DPP read-after-VALU-write hazards (and count the s_nop wait
states that are not needed).

    python asmpass/dpp_hazards.py <file.s> [--kernel SUBSTR]

The rule (CDNA3 ISA, "manually inserted wait states"): a DPP instruction that reads a VGPR
needs two wait states after a VALU instruction that wrote that VGPR.  Checked here for
every source operand (src0, the DPP-read one, and src1), but not for a v_fmac's tied
accumulator: the engine's v_fmac_f64_dpp chains (bdot12 & co.) forward the accumulator from
one instruction to the next with no wait state and are bit-exact against the oracle, so the
hardware interlocks that operand (LLVM's checkDPPHazards would also count it).  Every instruction issued in between counts as one wait
state, `s_nop N` as N + 1.  The scan is linear within basic blocks (a label resets nothing:
it assumes the worst, that the predecessor's last instructions immediately precede), which
is conservative at block boundaries.  The EXEC rule is checked the same way: a DPP
instruction needs five wait states after a VALU write of EXEC (v_cmpx, or a VALU with EXEC
as its destination).  v_permlane* and v_swap* write both of their operands.  Exit status 1
if a hazard is found.
"""
import argparse
import re
import sys

VREG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")


def regs(tok):
    out = set()
    for m in VREG.finditer(tok):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def valu_writes(op, args):
    """(VGPRs, EXEC?) a VALU instruction writes; (set(), False) for anything else."""
    if not op.startswith("v_") or op.startswith(("v_readfirstlane", "v_readlane")):
        return set(), False
    ops = args.split(",")
    dst = ops[0].strip()
    if op.startswith("v_cmp"):  # writes an SGPR pair / VCC, or EXEC (v_cmpx)
        return set(), op.startswith("v_cmpx") or dst.startswith("exec")
    wrote = regs(dst)
    if op.startswith(("v_permlane", "v_swap")) and len(ops) > 1:  # both operands are written
        wrote |= regs(ops[1])
    return wrote, dst.startswith("exec")


def scan(lines):
    """Yields (line_no, text, needed, available) for every DPP instruction, where
    available = wait states since the last VALU write of its DPP source (capped at 3),
    needed 2; or, where a VALU write of EXEC is fewer than five wait states back, that
    count with needed 5."""
    hist = []  # (wait states this instruction provides, VGPRs it wrote if VALU, EXEC written)
    for no, raw in lines:
        s = raw.split(";")[0].strip()
        if not s or s.endswith(":") or s.startswith("."):
            continue
        op = s.split()[0]
        args = s[len(op):]
        if "_dpp" in op:
            ops = [a.strip() for a in args.split(",")]
            need = set()  # the VGPRs of every source (src0 is the DPP-read one)
            for o in ops[1:]:
                need |= regs(o.split()[0])
            ws = 0
            avail = 3
            for provided, wrote, _ in reversed(hist[-4:]):
                if wrote & need:
                    avail = ws
                    break
                ws += provided
                if ws >= 3:
                    break
            ws = 0
            avail_x = 5
            for provided, _, wx in reversed(hist[-6:]):
                if wx:
                    avail_x = ws
                    break
                ws += provided
                if ws >= 5:
                    break
            yield (no, s, 5, avail_x) if avail_x < 5 else (no, s, 2, avail)
        wrote, wexec = valu_writes(op, args)
        provided = int(s.split()[1]) + 1 if op == "s_nop" else 1
        hist.append((provided, wrote, wexec))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="engine_kernel")
    a = ap.parse_args()
    text = open(a.asm).read().splitlines()
    # the functions whose name contains the substring
    funcs, cur = [], None
    for i, l in enumerate(text):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            cur = m.group(1) if a.kernel in m.group(1) else None
            if cur:
                funcs.append((cur, []))
        if cur and funcs:
            funcs[-1][1].append((i + 1, l))
        if l.startswith(".Lfunc_end"):
            cur = None
    bad = 0
    for name, lines in funcs:
        n = tight = 0
        for no, s, need, avail in scan(lines):
            n += 1
            if avail < need:
                bad += 1
                print(f"HAZARD {name} line {no}: {s} (only {avail} wait states)")
            elif avail == need:
                tight += 1
        print(f"{name}: {n} DPP instructions, {tight} with exactly the 2 wait states they need")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
