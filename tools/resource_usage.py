#!/usr/bin/env python3
"""The compiler's register / scratch / LDS budget per engine kernel instantiation.

    python tools/resource_usage.py [--horizons 16 32 48 64] [--extra -DMPCQ_CR]

Compiles mpcq_engine.hip for each horizon with -Rpass-analysis=kernel-resource-usage
(the production flags of the Makefile) and writes profiles/resource_usage.json:
{N: {kernel: {VGPRs, AGPRs, SGPRs, ScratchSize, VGPR spill, SGPR spill, Occupancy,
LDS}}}.  tools/prof_summary.py quotes it next to the rocprofv3 trace's register
fields (the trace reports the hardware allocation granule, not the compiler's count).
"""
import argparse
import json
import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "mpc-tsid_amd", "csrc")
KIND = {"ELb1ELb1ELb0EE": "fused solve (production)", "ELb1ELb1ELb1EE": "fused solve + polish",
        "ELb0ELb1ELb0EE": "qp_solve", "ELb0ELb1ELb1EE": "qp_solve + polish", "ELb1ELb0ELb0EE": "formulation only"}


def usage(N, extra=()):
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function"]
    if N != 40:
        flags += ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]  # as the Makefile
    cmd = ["/opt/rocm/bin/hipcc", *flags, *extra, f"-DMPCQ_ENGINE_N={N}", "-c", "-o", f"/tmp/ru_{N}.o",
           os.path.join(CSRC, "mpcq_engine.hip"), "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
    res, cur = {}, None
    for line in out.splitlines():
        m = re.search(r"remark: +Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            kind = next((v for k, v in KIND.items() if k in name), name)
            cur = res.setdefault(kind, {})
            continue
        m = re.search(r"remark: +([A-Za-z ]+?)(?: \[[a-z/A-Z]+\])?: (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--horizons", type=int, nargs="+", default=[16, 32, 48, 64])
    ap.add_argument("--extra", nargs="*", default=[])
    a = ap.parse_args()
    out = {str(N): usage(N, a.extra) for N in a.horizons}
    path = os.path.join(REPO, "profiles", "resource_usage.json")
    json.dump(out, open(path, "w"), indent=1)
    for N, ks in out.items():
        p = ks.get("fused solve (production)", {})
        print(f"N={N}: production VGPRs {p.get('VGPRs')} AGPRs {p.get('AGPRs')} scratch {p.get('ScratchSize')} B/lane "
              f"VGPR spill {p.get('VGPRs Spill')} occupancy {p.get('Occupancy')} waves/SIMD, LDS {p.get('LDS Size')} B")


if __name__ == "__main__":
    main()
