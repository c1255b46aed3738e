"""Per-iteration time at every horizon of a range, one library variant per process.

    [MPCQ_LIB_VARIANT=exp:<name>] python tools/bigsweep.py [--Ns 33-64] [--iters 1000]

256 copies of instance 0 of a seeded trot batch (one per CU), adaptive rho off and
eps ~0 so every copy runs exactly `iters` iterations with OSQP's check every 25:
kernel time / iters is the per-iteration latency alone on a CU.  Used to choose, per
horizon beyond 32 stages, between register-allocation variants of the engine (a
timing experiment: the solver settings here are not the reference's).
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--Ns", default="33-64")
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    lo, _, hi = a.Ns.partition("-")
    Ns = range(int(lo), int(hi or lo) + 1)
    import torch
    import mpcq
    dev = torch.device("cuda", 0)
    B = 256
    tag = os.environ.get("MPCQ_LIB_VARIANT") or "prod"
    for N in Ns:
        src = mpcq.synth.make_batch(4, N, gaits=("trot",), seed=2)
        xr = torch.from_numpy(np.ascontiguousarray(np.repeat(src["xref"][:1], B, axis=0))).to(dev)
        fs = torch.from_numpy(np.ascontiguousarray(np.repeat(src["fsteps"][:1], B, axis=0))).to(dev)
        f0 = torch.empty((B, 12), dtype=torch.float64, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        it = torch.empty(B, dtype=torch.int32, device=dev)
        eng = mpcq.Engine(N, adaptive_rho=0, max_iter=a.iters, eps_abs=1e-30, eps_rel=1e-30)
        ms = []
        for _ in range(a.reps):
            eng.solve_device(B, xr.data_ptr(), fs.data_ptr(), f0.data_ptr(), st.data_ptr(), it.data_ptr())
            torch.cuda.synchronize()
            ms.append(eng.last_kernel_ms()[1])
        eng.close()
        m = float(np.median(ms))
        print(f"{tag} N={N:3d} {1e3 * m / int(it[0].item()):7.3f} us/iteration ({int(it[0].item())} iterations)", flush=True)


if __name__ == "__main__":
    main()
