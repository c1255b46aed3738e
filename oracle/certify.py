"""Exact optimum of each MPC QP, certified by its KKT conditions.

TEST INFRASTRUCTURE ONLY: used by tests/ and by bench.py's parity leg (after
the timed region) as the checker.  The product package never imports it.

Each instance's QP (MPC.py:98-288 formulation via oracle/mpcq_oracle.c, which
is pinned to A.data / l / u captured from the unmodified reference) is strictly
convex (P diagonal > 0, MPC.py:250-279), so its optimum x* is unique and is the
one target any OSQP run at eps 1e-7 (MPC.py:414-416) approximates.  x* is found
by primal-dual active-set steps on the UNSCALED KKT system with sparse LU and
iterative refinement, seeded with a solver's own (z, y) -- the same method
tests/golden/gen_golden.py uses for the committed fixtures, where it starts
from an ADMM warm phase instead -- and certified by its KKT residuals:
primal infeasibility, stationarity |P x + A' y|, multiplier signs and
complementarity.  A certificate below ~1e-9 pins x* independently of the
GPU code (which it only uses as a starting guess for the active set).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as sla

from . import oracle as O


def qp_data(xref, fsteps, mode: int = 0, params=None):
    """(P diag, A csc, l, u) of one instance, exactly as MPC.call_solver hands them to OSQP."""
    p = params or O.default_params()
    N = np.shape(xref)[1] - 1
    Ax, l, u = O.formulate(xref, fsteps, mode, p)
    indptr, indices = O.pattern(N)
    n, m, _ = O.dims(N)
    A = sp.csc_matrix((Ax, indices, indptr), shape=(m, n))
    w = np.array(list(p.state_weights))
    Pd = np.concatenate([np.tile(w, N), np.full(12 * N, p.force_weight)])
    return Pd, A, l, u


def kkt_residuals(Pd, A, l, u, x, y):
    """(primal infeasibility, stationarity, multiplier-sign violation, complementarity)."""
    z = A @ x
    prim = max(np.maximum(l - z, 0).max(), np.maximum(z - u, 0).max())
    stat = np.abs(Pd * x + A.T @ y).max()
    lo_gap = np.where(np.isfinite(l), z - l, np.inf)
    hi_gap = np.where(np.isfinite(u), u - z, np.inf)
    sign = max(np.maximum(y, 0)[hi_gap > 1e-9].max(initial=0.0),
               np.maximum(-y, 0)[lo_gap > 1e-9].max(initial=0.0))
    comp = max((np.maximum(-y, 0) * np.minimum(lo_gap, 1e3)).max(),
               (np.maximum(y, 0) * np.minimum(hi_gap, 1e3)).max())
    return np.array([prim, stat, sign, comp])


def _eq_solve(Pd, A, l, u, lo, hi, delta=1e-9, refine=30):
    n, m = A.shape[1], A.shape[0]
    act = lo | hi
    Aa = A[act]
    b = np.where(lo, l, u)[act]
    ma = Aa.shape[0]
    K = sp.bmat([[sp.diags(Pd + delta), Aa.T], [Aa, -delta * sp.eye(ma)]]).tocsc()
    K0 = sp.bmat([[sp.diags(Pd), Aa.T], [Aa, None]]).tocsc()
    F = sla.splu(K)
    rhs = np.concatenate([np.zeros(n), b])
    sol = F.solve(rhs)
    for _ in range(refine):
        d = F.solve(rhs - K0 @ sol)
        sol = sol + d
        if np.abs(d).max() <= 1e-17 * max(1.0, np.abs(sol).max()):
            break
    yp = np.zeros(m)
    yp[act] = sol[n:]
    return sol[:n], yp


def exact_optimum(Pd, A, l, u, x0, y0, rounds: int = 40):
    """Active-set refinement from a solver point (x0, y0); returns (x*, y*, kkt residuals)."""
    A = A.tocsc()
    z0 = A @ x0
    rownz = np.diff(A.tocsr().indptr) > 0
    eq = (u - l) < 1e-12
    lo = (z0 - l < -y0) & rownz
    hi = (~lo) & (u - z0 < y0) & rownz
    lo |= eq & rownz & ~hi
    best = None
    seen = set()
    for _ in range(rounds):
        key = (lo.tobytes(), hi.tobytes())
        if key in seen:
            break
        seen.add(key)
        xp, yp = _eq_solve(Pd, A, l, u, lo, hi)
        res = kkt_residuals(Pd, A, l, u, xp, yp)
        if best is None or res.max() < best[2].max():
            best = (xp, yp, res)
        if res.max() < 1e-13:
            break
        zp = A @ xp
        tol = 1e-12
        keep_lo = lo & ((yp <= tol) | eq)
        keep_hi = hi & ((yp >= -tol) | eq)
        add_lo = (zp < l - tol) & rownz & ~keep_hi
        add_hi = (zp > u + tol) & rownz & ~keep_lo
        lo, hi = keep_lo | add_lo, keep_hi | add_hi
    return best


def certified_forces(xref, fsteps, x, y, mode: int = 0, params=None, tol: float = 1e-9):
    """For a batch: f0* (B, 12), the KKT residual max per instance and a certified mask.

    (x, y) are a solver's primal / dual outputs (OSQP's unscaled convention,
    y > 0 on active upper bounds); they only seed the active set."""
    xref = np.asarray(xref)
    B = xref.shape[0]
    N = xref.shape[2] - 1
    f0 = np.full((B, 12), np.nan)
    kkt = np.full(B, np.inf)
    for b in range(B):
        Pd, A, l, u = qp_data(xref[b], fsteps[b], mode, params)
        l = np.maximum(l, -1e30)
        xs, ys, res = exact_optimum(Pd, A, l, u, x[b], y[b])
        f0[b] = xs[12 * N:12 * N + 12]
        kkt[b] = res.max()
    return f0, kkt, kkt < tol
