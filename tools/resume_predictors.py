"""Which quantity at suspension ranks a sliced C3 solve's remaining work?  (DESIGN.md section 8,
sliced solves: the order of the resumed launches.)  CPU only.

    python tools/resume_predictors.py [--K 1600]

The C3 batch (seed 2, trot, N = 32): the oracle's full iteration counts, then for every instance
still iterating after K iterations (the ones a slice of K suspends) the oracle's restatement
run to max_iter = K: the unscaled primal / dual residuals, their relative forms, rho and the
primal / dual ratio, each correlated (Spearman) with the final iteration count.
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mpc-tsid_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=1600)
    a = ap.parse_args()
    import scipy.sparse as sp
    from scipy.stats import spearmanr
    import mpcq
    from oracle import oracle as O
    O.build()
    N, B, K = 32, 1024, a.K
    b = mpcq.synth.make_batch(B, N, gaits=("trot",), seed=2)
    t = time.time()
    full = O.solve_batch(b["xref"], b["fsteps"], 0, nthreads=os.cpu_count() or 1)["iters"]
    print(f"C3 batch: oracle {time.time() - t:.1f} s, iterations median {np.median(full):.0f} max {full.max()}")
    sel = np.where(full > K)[0]
    print(f"suspended at K = {K}: {len(sel)} instances, their final iterations median {np.median(full[sel]):.0f} "
          f"max {full[sel].max()}")
    indptr, indices = O.pattern(N)
    n, m, _ = O.dims(N)
    p0 = O.default_params()
    Pd = np.concatenate([np.tile(np.array(p0.state_weights), N), np.full(12 * N, p0.force_weight)])
    p = O.default_params(max_iter=K)
    F = {k: np.zeros(len(sel)) for k in ("r_prim", "r_dual", "r_prim_rel", "r_dual_rel", "rho", "log_prim_over_dual")}
    for j, i in enumerate(sel):
        Ax, l, u = O.formulate(b["xref"][i], b["fsteps"][i])
        A = sp.csc_matrix((Ax, indices, indptr), shape=(m, n))
        r = O.qp_solve(N, Ax, l, u, params=p)
        x, y = r["x"], r["y"]
        ax, aty = A @ x, A.T @ y
        F["r_prim"][j] = np.max(np.maximum(0.0, np.maximum(l - ax, ax - u)))
        F["r_dual"][j] = np.max(np.abs(Pd * x + aty))
        F["r_prim_rel"][j] = F["r_prim"][j] / max(np.max(np.abs(ax)), 1e-300)
        F["r_dual_rel"][j] = F["r_dual"][j] / max(np.max(np.abs(Pd * x)), np.max(np.abs(aty)), 1e-300)
        F["rho"][j] = r["rho"]
        F["log_prim_over_dual"][j] = np.log(F["r_prim"][j] + 1e-30) - np.log(F["r_dual"][j] + 1e-30)
    for k, v in F.items():
        print(f"K = {K}  {k:20s} Spearman with the final iteration count {spearmanr(v, full[sel])[0]:+.3f}")


if __name__ == "__main__":
    main()
