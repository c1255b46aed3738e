"""Can a short prefix of the solve rank a cold batch by its final iteration count?
  CPU only.

    python tools/early_predictors.py [--K 50 100 150]

For every instance of the C2 batch (seed 2, trot, N = 16) the oracle's OSQP restatement
runs max_iter = K iterations; the unscaled primal residual (box violation of A x), the
dual residual ||P x + A'y||, their relative forms and the rho reached are correlated
(Spearman) with the full solve's iteration count.
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mpc-tsid_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, nargs="+", default=[50, 100, 150, 200])
    a = ap.parse_args()
    import scipy.sparse as sp
    from scipy.stats import spearmanr
    import mpcq
    from oracle import oracle as O
    O.build()
    N, B = 16, 1024
    b = mpcq.synth.make_batch(B, N, gaits=("trot",), seed=2)
    full = O.solve_batch(b["xref"], b["fsteps"], 0, nthreads=os.cpu_count() or 1)["iters"]
    indptr, indices = O.pattern(N)
    n, m, _ = O.dims(N)
    p0 = O.default_params()
    Pd = np.concatenate([np.tile(np.array(p0.state_weights), N), np.full(12 * N, p0.force_weight)])
    qps = [O.formulate(b["xref"][i], b["fsteps"][i]) for i in range(B)]
    for K in a.K:
        p = O.default_params(max_iter=K)
        F = {k: np.zeros(B) for k in ("r_prim", "r_dual", "r_prim_rel", "r_dual_rel", "rho")}
        for i, (Ax, l, u) in enumerate(qps):
            A = sp.csc_matrix((Ax, indices, indptr), shape=(m, n))
            r = O.qp_solve(N, Ax, l, u, params=p)
            x, y = r["x"], r["y"]
            ax, aty = A @ x, A.T @ y
            F["r_prim"][i] = np.max(np.maximum(0.0, np.maximum(l - ax, ax - u)))
            F["r_dual"][i] = np.max(np.abs(Pd * x + aty))
            F["r_prim_rel"][i] = F["r_prim"][i] / max(np.max(np.abs(ax)), 1e-300)
            F["r_dual_rel"][i] = F["r_dual"][i] / max(np.max(np.abs(Pd * x)), np.max(np.abs(aty)), 1e-300)
            F["rho"][i] = r["rho"]
        for k, v in F.items():
            rho = spearmanr(v, full)[0] if np.ptp(v) > 0 else float("nan")
            print(f"K = {K:4d}  {k:12s} Spearman {rho:+.3f}", flush=True)


if __name__ == "__main__":
    main()
