#!/usr/bin/env python3
"""hipcc -c with the nop-elision pass (nop_elide.py) between the device compiler and
the device assembler:

    python asmpass/hipcc_elide.py <hipcc args ... -c -o out.o src>   (Makefile: the engine units)

Replays the driver's own job list (`hipcc -### -save-temps`) in a scratch directory; after
the device `-S` job it rewrites the gfx950 assembly with nop_elide and re-scans it with
dpp_hazards (exit 1 on a hazard), then runs the remaining jobs (device assembler, device
link, offload bundle, host compile) unchanged."""
import os
import shlex
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dpp_hazards  # noqa: E402
import nop_elide  # noqa: E402


def main():
    args = sys.argv[1:]
    out = os.path.abspath(args[args.index("-o") + 1])
    args = [os.path.abspath(a) if os.path.exists(a) and not a.startswith("-") else a for a in args]
    args[args.index("-o") + 1] = out
    with tempfile.TemporaryDirectory() as tmp:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "-###", "-save-temps"] + args, cwd=tmp,
                           capture_output=True, text=True, check=True)
        jobs = [shlex.split(l) for l in r.stderr.splitlines() if l.startswith(' "')]
        for job in jobs:
            subprocess.run(job, cwd=tmp, check=True)
            if "-S" in job and "amdgcn-amd-amdhsa" in job[job.index("-triple") + 1]:
                s = os.path.join(tmp, job[job.index("-o") + 1])
                lines = open(s).read().split("\n")
                el, removed, kept = nop_elide.elide(lines)
                open(s, "w").write("\n".join(el))
                bad = sum(1 for no, t, need, av in dpp_hazards.scan(enumerate(el, 1)) if av < need)
                print(f"{os.path.basename(out)}: nop_elide {removed} removed, {kept} kept; "
                      f"{bad} DPP hazards after")
                if bad:
                    sys.exit(1)


if __name__ == "__main__":
    main()
