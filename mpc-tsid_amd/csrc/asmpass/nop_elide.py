#!/usr/bin/env python3
"""Drop the `s_nop 1` that opens the engine's v_fmac_f64_dpp inline-asm blocks where the
compiler's schedule already separates the block from every write it depends on.

    python asmpass/nop_elide.py <in.s> <out.s>   (the build runs it through hipcc_elide.py)

The asm blocks (bdot12, fmac3_bc, the Gauss-Jordan and Schur macros, the colF fold) start
with `s_nop 1` because a VALU write of a VGPR followed by a DPP read of it needs two wait
states, and inline asm cannot know what the compiler schedules before it.  In the compiled
program most of those nops follow instructions that write nothing the block reads.  This
pass removes such a nop when all of the following hold (conservative on purpose):
  - the nop is the first instruction of an inline-asm region (;;#ASMSTART) and is exactly
    `s_nop 1`;
  - the two instructions issued before it (an earlier asm region's included: its text is
    what is issued) are ordinary instructions (no label, no branch, no s_nop) and neither writes a VGPR that any
    instruction of the region reads (covers the DPP-source rule, 2 wait states, and the
    transcendental-result rule, 1 wait state);
  - no VALU write of EXEC (v_cmpx) within the 5 instructions before it (DPP after an EXEC
    write needs 5 wait states); a label met in that walk ends it only where the program has
    no VALU write of EXEC anywhere (a branch from elsewhere could otherwise arrive right
    after one); else the nop stays;
  - the kernel has no MFMA (their result hazards are longer).
After the pass, dpp_hazards.py re-scans the output and the build fails on any
hazard.  Prints the count of nops kept and removed."""
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from dpp_hazards import regs, valu_writes  # noqa: E402


def instr(line):
    s = line.split(";")[0].strip()
    if not s or s.startswith("."):
        return None
    return s


def written(s):
    """VGPRs a VALU instruction writes (v_permlane / v_swap: both operands)."""
    op = s.split()[0]
    return valu_writes(op, s[len(op):])[0]


def writes_exec(s):
    op = s.split()[0]
    return valu_writes(op, s[len(op):])[1]


def elide(lines):
    if any("v_mfma" in l for l in lines):
        return lines, 0, sum(1 for l in lines if l.strip() == "s_nop 1")
    out = list(lines)
    removed = kept = 0
    any_exec = any(instr(l) and writes_exec(instr(l)) for l in lines)
    i = 0
    n = len(lines)
    while i < n:
        if lines[i].strip() != ";;#ASMSTART":
            i += 1
            continue
        # the region's instructions
        j = i + 1
        body = []
        while j < n and lines[j].strip() != ";;#ASMEND":
            body.append(j)
            j += 1
        first = [k for k in body if instr(lines[k])]
        if not first or instr(lines[first[0]]) != "s_nop 1":
            i = j
            continue
        reads = set()
        for k in first[1:]:
            s = instr(lines[k])
            op = s.split()[0]
            for a in s[len(op):].split(",")[1:]:
                reads |= regs(a.split()[0] if a.strip() else a)
            if op.startswith("v_fmac") or op.startswith("v_fma"):  # the accumulator is read too
                reads |= regs(s[len(op):].split(",")[0])
        # walk back over the issued instructions before the region
        ok = True
        seen = 0
        k = i - 1
        while k >= 0 and seen < 5:
            raw = lines[k].strip()
            if raw in (";;#ASMSTART", ";;#ASMEND"):  # an earlier region's text is literal
                k -= 1
                continue
            if raw.split(";")[0].strip().endswith(":"):  # a label (a branch target)
                if seen < 2 or any_exec:
                    ok = False
                break
            s = instr(lines[k])
            if s is None:
                k -= 1
                continue
            op = s.split()[0]
            if writes_exec(s):
                ok = False
                break
            if seen < 2:
                if op.startswith(("s_nop", "s_cbranch", "s_branch", "s_setpc", "s_swappc")):
                    ok = False
                    break
                if written(s) & reads:
                    ok = False
                    break
            seen += 1
            k -= 1
        if ok:
            out[first[0]] = "\t; s_nop 1 elided (tools/nop_elide.py)"
            removed += 1
        else:
            kept += 1
        i = j
    return out, removed, kept


def main():
    src, dst = sys.argv[1], sys.argv[2]
    lines = open(src).read().split("\n")
    out, removed, kept = elide(lines)
    open(dst, "w").write("\n".join(out))
    print(f"nop_elide: {removed} removed, {kept} kept")


if __name__ == "__main__":
    main()
