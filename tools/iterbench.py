"""Per-iteration latency of the production kernel, free of the batch's tail effects.

    python tools/iterbench.py [--N 16] [--reps 5] [--polish]

Takes the C2 batch (bench.py's seeded synthetic instances), finds its slowest
instance and launches B identical copies of it (B = 256: one instance per CU;
512: two, the bench's occupancy; 1024: two resident, two rounds).  Every copy
runs the same iterations, so kernel time / iterations is the per-iteration
latency at that occupancy.
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pick", choices=("slowest", "fastest"), default="slowest",
                    help="which instance of the batch to copy")
    ap.add_argument("--polish", action="store_true", help="the bench's accuracy mode (polish=2 instantiation)")
    ap.add_argument("--batches", type=int, nargs="+", default=[256, 512, 1024],
                    help="copies per launch (below 256 some CUs idle: the per-instance share of each XCD's L2 grows)")
    a = ap.parse_args()
    import torch
    import mpcq
    dev = torch.device("cuda", 0)
    eng = mpcq.Engine(a.N, **(dict(polish=2, polish_rounds=8, polish_refine_iter=10) if a.polish else {}))
    src = mpcq.synth.make_batch(1024, a.N, gaits=("trot",), seed=2)  # bench.py C2 data

    def run(xref, fsteps, reps):
        B = xref.shape[0]
        xr = torch.from_numpy(np.ascontiguousarray(xref)).to(dev)
        fs = torch.from_numpy(np.ascontiguousarray(fsteps)).to(dev)
        f0 = torch.empty((B, 12), dtype=torch.float64, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        it = torch.empty(B, dtype=torch.int32, device=dev)
        ms = []
        for _ in range(reps):
            eng.solve_device(B, xr.data_ptr(), fs.data_ptr(), f0.data_ptr(), st.data_ptr(), it.data_ptr())
            torch.cuda.synchronize()
            ms.append(eng.last_kernel_ms()[1])
        return it.cpu().numpy(), float(np.median(ms))

    its, ms = run(src["xref"], src["fsteps"], a.reps)
    slow = int(np.argmax(its)) if a.pick == "slowest" else int(np.argmin(its))
    r = eng.solve(src["xref"][slow:slow + 1], src["fsteps"][slow:slow + 1])
    print(f"C2 batch: kernel {ms:.3f} ms, iterations median {np.median(its):.0f} max {its.max()} ({a.pick}: instance {slow}, "
          f"{int(r['rho_updates'][0])} rho updates)")
    for B in a.batches:
        xr = np.repeat(src["xref"][slow:slow + 1], B, axis=0)
        fs = np.repeat(src["fsteps"][slow:slow + 1], B, axis=0)
        it2, ms2 = run(xr, fs, a.reps)
        assert (it2 == it2[0]).all()
        n_it = int(it2[0])
        print(f"B={B:5d} copies of the slowest: {ms2:8.3f} ms, {n_it} iterations, "
              f"{1e3 * ms2 / n_it:7.3f} us/iteration")
    eng.close()


if __name__ == "__main__":
    main()
