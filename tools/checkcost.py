"""Cost of one termination check / rho-adaptation step, measured on the production kernel.

    python tools/checkcost.py [--N 16]

Runs 256 copies of one C2 instance (one per CU) with adaptive rho off and
max_iter fixed, so every configuration runs exactly max_iter iterations, and
varies check_termination: the time difference per check is the check's cost on
the critical path.  (A timing experiment only: the solver settings here are not
the reference's.)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=16)
    ap.add_argument("--iters", type=int, default=2000)
    a = ap.parse_args()
    import torch
    import mpcq
    dev = torch.device("cuda", 0)
    src = mpcq.synth.make_batch(1024, a.N, gaits=("trot",), seed=2)
    B, iters = 256, a.iters
    xr = torch.from_numpy(np.ascontiguousarray(np.repeat(src["xref"][:1], B, axis=0))).to(dev)
    fs = torch.from_numpy(np.ascontiguousarray(np.repeat(src["fsteps"][:1], B, axis=0))).to(dev)
    f0 = torch.empty((B, 12), dtype=torch.float64, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    base = None
    for chk in (0, 100, 25, 5):
        eng = mpcq.Engine(a.N, adaptive_rho=0, max_iter=iters, check_termination=chk, eps_abs=1e-30, eps_rel=1e-30)
        ms = []
        for _ in range(5):
            eng.solve_device(B, xr.data_ptr(), fs.data_ptr(), f0.data_ptr(), st.data_ptr(), it.data_ptr())
            torch.cuda.synchronize()
            ms.append(eng.last_kernel_ms()[1])
        m = float(np.median(ms))
        n_it = int(it[0].item())
        n_chk = iters // chk if chk else 0
        if base is None:
            base = m
        extra = (m - base) / n_chk * 1e3 if n_chk else 0.0
        print(f"check every {chk:4d}: {m:8.3f} ms, {n_it} iterations, {1e3 * m / n_it:6.3f} us/iteration, "
              f"{n_chk} checks, {extra:6.2f} us per check", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
