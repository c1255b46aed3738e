"""Which quantity at suspension ranks a sliced C3 solve's remaining work?  (DESIGN.md section 8,
sliced solves: the order of the resumed launches.)  CPU only.

    python tools/resume_predictors.py [--K 1200 1600]

The C3 batch (seed 2, trot, N = 32): the oracle's full iteration counts, then for every instance
still iterating after K iterations (the ones a slice of K suspends) the oracle's restatement
run to max_iter = K (and K / 2): the unscaled primal / dual residuals, their relative forms,
rho, the primal / dual ratio, and the iterations left extrapolated from the relative primal
residual's geometric decay between K / 2 and K (what the engine's key does, with each residual
over its own tolerance), each correlated (Spearman) with the final iteration count.
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
    ap.add_argument("--K", type=int, nargs="+", default=[1200, 1600])
    a = ap.parse_args()
    import scipy.sparse as sp
    from scipy.stats import spearmanr
    import mpcq
    from oracle import oracle as O
    O.build()
    N, B = 32, 1024
    b = mpcq.synth.make_batch(B, N, gaits=("trot",), seed=2)
    t = time.time()
    full = O.solve_batch(b["xref"], b["fsteps"], 0, nthreads=os.cpu_count() or 1)["iters"]
    print(f"C3 batch: oracle {time.time() - t:.1f} s, iterations median {np.median(full):.0f} max {full.max()}")
    indptr, indices = O.pattern(N)
    n, m, _ = O.dims(N)
    p0 = O.default_params()
    Pd = np.concatenate([np.tile(np.array(p0.state_weights), N), np.full(12 * N, p0.force_weight)])
    qps = {}

    def at(i, K):
        if i not in qps:
            Ax, l, u = O.formulate(b["xref"][i], b["fsteps"][i])
            qps[i] = (Ax, l, u, sp.csc_matrix((Ax, indices, indptr), shape=(m, n)))
        Ax, l, u, A = qps[i]
        r = O.qp_solve(N, Ax, l, u, params=O.default_params(max_iter=K))
        x, y = r["x"], r["y"]
        ax, aty = A @ x, A.T @ y
        rp = np.max(np.maximum(0.0, np.maximum(l - ax, ax - u)))
        rd = np.max(np.abs(Pd * x + aty))
        return dict(r_prim=rp, r_dual=rd, r_prim_rel=rp / max(np.max(np.abs(ax)), 1e-300),
                    r_dual_rel=rd / max(np.max(np.abs(Pd * x)), np.max(np.abs(aty)), 1e-300), rho=r["rho"],
                    log_prim_over_dual=np.log(rp + 1e-30) - np.log(rd + 1e-30))

    for K in a.K:
        sel = np.where(full > K)[0]
        print(f"suspended at K = {K}: {len(sel)} instances, their final iterations median "
              f"{np.median(full[sel]):.0f} max {full[sel].max()}")
        F2 = [at(i, K) for i in sel]
        F1 = [at(i, K // 2) for i in sel]
        for k in F2[0]:
            v = np.array([f[k] for f in F2])
            print(f"K = {K}  {k:24s} Spearman with the final iteration count {spearmanr(v, full[sel])[0]:+.3f}")
        r2 = np.array([f["r_prim_rel"] for f in F2])
        r1 = np.array([f["r_prim_rel"] for f in F1])
        eps = 1e-7  # (the relative primal tolerance scale: eps_rel; the engine divides by eps_pri itself)
        left = np.where(r1 > r2, np.log(np.maximum(r2 / eps, 1.0)) / np.log(r1 / np.maximum(r2, 1e-300)) * (K - K // 2),
                        1e30)
        print(f"K = {K}  {'extrapolated_left':24s} Spearman with the final iteration count "
              f"{spearmanr(left, full[sel])[0]:+.3f}")


if __name__ == "__main__":
    main()
