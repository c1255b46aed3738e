#!/usr/bin/env python3
"""The gfx950 code objects inside a built library, and their disassembly.

    python asmpass/codeobj.py <libmpcq.so> [--scan]

A HIP shared library carries its device code in the `.hip_fatbin` section: one clang
offload bundle per compiled unit ("__CLANG_OFFLOAD_BUNDLE__", a count, then per entry
offset / size / target triple), 4096-aligned one after the other.  extract() returns the
amdgcn ELF code objects; disassemble() runs llvm-objdump on one.  --scan runs
dpp_hazards.scan over every kernel of the shipped library (what the build checked on its
assembly, re-checked on the binary)."""
import os
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def fatbin(so_path):
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={out}", so_path, os.devnull],
                       check=True, capture_output=True)
        with open(out, "rb") as f:
            return f.read()


def extract(so_path, target="gfx950"):
    """[(bundle index, code object bytes)] for every amdgcn entry built for `target`."""
    blob = fatbin(so_path)
    objs = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + len(MAGIC))[0]
        q = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, q)
            triple = blob[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if "amdgcn" in triple and triple.endswith(target):
                objs.append((len(objs), blob[pos + off:pos + off + size]))
        pos = blob.find(MAGIC, pos + len(MAGIC))
    return objs


def disassemble(code, mcpu="gfx950"):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code)
        f.flush()
        r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--mcpu={mcpu}", "--no-show-raw-insn", f.name],
                           check=True, capture_output=True, text=True)
    return r.stdout


def kernels(text):
    """{symbol: [(line_no, instruction text)]} from llvm-objdump output ("//" comments
    dropped; a function starts at a "<symbol>:" line)."""
    out, cur = {}, None
    for i, line in enumerate(text.splitlines(), 1):
        s = line.split("//")[0].rstrip()
        if s.endswith(">:") and "<" in s:
            cur = s[s.index("<") + 1:-2]
            out[cur] = []
        elif cur is not None and s.strip():
            out[cur].append((i, s.strip()))
    return out


def main():
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import dpp_hazards
    so = sys.argv[1]
    objs = extract(so)
    bad = nk = ndpp = 0
    for idx, code in objs:
        for name, lines in kernels(disassemble(code)).items():
            nk += 1
            for no, s, need, av in dpp_hazards.scan(lines):
                ndpp += 1
                if av < need:
                    bad += 1
                    print(f"HAZARD object {idx} {name} line {no}: {s}")
    print(f"{len(objs)} gfx950 code objects, {nk} functions, {ndpp} DPP instructions, {bad} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
