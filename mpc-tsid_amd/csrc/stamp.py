#!/usr/bin/env python3
"""The library's build stamp (include/mpcq.h mpcq_build_info, "src_sha256=<16 hex>").

    python3 stamp.py ["HIPFLAGS=... SCHED=... ELIDE=..."]   (the Makefile's call)

First 16 hex digits of sha256 over every input that changes the shipped code: the HIP
sources (csrc/*.hip, name order), the assembly pass (asmpass/hipcc_elide.py, nop_elide.py,
dpp_hazards.py), the Makefile, the headers (mpcq_internal.h: LaunchArgs and the workspace
layout; include/mpcq.h), the C++ units (csrc/*.cpp, name order), then the effective
compiler flags as one string.  Without an argument the flags are the Makefile's defaults,
so mpcq.source_sha() (mpcq/_lib.py) and a default `make` agree; a build with overridden
flags carries another stamp, and bench.py then drops PMC figures profiled on the default
build (profiles/pmc_traffic.json)."""
import hashlib
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ELIDE_PASS = ("hipcc_elide.py", "nop_elide.py", "dpp_hazards.py")


def inputs(csrc: str = HERE):
    names = sorted(n for n in os.listdir(csrc) if n.endswith(".hip"))
    names += [os.path.join("asmpass", n) for n in ELIDE_PASS]
    names += ["Makefile", "mpcq_internal.h", os.path.join("..", "..", "include", "mpcq.h")]
    names += sorted(n for n in os.listdir(csrc) if n.endswith(".cpp"))
    return [os.path.join(csrc, n) for n in names]


def default_flags(csrc: str = HERE) -> str:
    """The flag string a plain `make` hashes, read from the Makefile's defaults."""
    text = open(os.path.join(csrc, "Makefile")).read()

    def var(name, op):
        m = re.search(rf"^{name} {re.escape(op)} (.*)$", text, re.M)
        return m.group(1).strip() if m else ""
    arch = var("ARCH", "?=")
    hip = var("HIPFLAGS", "?=").replace("$(ARCH)", arch)
    return f"HIPFLAGS={hip} SCHED={var('SCHED', ':=')} ELIDE={var('ELIDE', '?=')}"


def stamp(csrc: str = HERE, flags: str | None = None) -> str:
    h = hashlib.sha256()
    for path in inputs(csrc):
        with open(path, "rb") as f:
            h.update(f.read())
    h.update((default_flags(csrc) if flags is None else flags).encode())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(stamp(HERE, sys.argv[1] if len(sys.argv) > 1 else None))
