"""CPU: the factorisation's Gauss-Jordan inverse with lazy pivot rows (mpcq_engine.hip
gj_step / gj12, kGjLazy, round 5) restated in numpy next to the normalised form it replaced.

The engine keeps one row of the 12 x 12 SPD block per lane; a pivot step updates every other
row with the broadcast pivot row.  Normalised: the pivot row becomes p / d at its step.
Lazy: the pivot lane's multiplier is 0 (its row stays p, its diagonal becomes 1) and every
row is scaled by its own pivot's 1/d after the twelfth step.  Both must give the inverse.
The engine runs them in FP64 with fused multiply-adds; numpy here rounds each product, so
the check is to the matrix's conditioning, not bit for bit."""
import numpy as np
import pytest


def gj_normalised(A):
    R = A.astype(np.float64).copy()
    n = R.shape[0]
    for k in range(n):
        d = R[k, k]
        idv = 1.0 / d
        p = R[k].copy()
        a = -R[:, k] * idv
        a[k] = idv
        base = R.copy()
        base[k] = 0.0
        R = base + np.outer(a, p)
        R[:, k] = a
    return R


def gj_lazy(A):
    R = A.astype(np.float64).copy()
    n = R.shape[0]
    sc = np.ones(n)
    for k in range(n):
        d = R[k, k]
        idv = 1.0 / d
        p = R[k].copy()
        a = -R[:, k] * idv
        a[k] = 0.0  # the pivot row stays p (its lane's multiplier is 0)
        col = a.copy()
        col[k] = 1.0  # ... and its diagonal 1: the row is d times the textbook row
        R = R + np.outer(a, p)
        R[:, k] = col
        sc[k] = idv
    return R * sc[:, None]


def spd(rng, n=12, cond=1e6):
    q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    ev = np.logspace(0, np.log10(cond), n)
    return (q * ev) @ q.T


@pytest.mark.parametrize("cond", [1e2, 1e6, 1e9])
def test_lazy_pivot_rows_invert(cond):
    rng = np.random.default_rng(7)
    for _ in range(20):
        A = spd(rng, cond=cond)
        ref = np.linalg.inv(A)
        lazy, norm = gj_lazy(A), gj_normalised(A)
        scale = np.abs(ref).max()
        tol = 1e-15 * cond * 50
        assert np.abs(lazy - ref).max() / scale < tol
        assert np.abs(norm - ref).max() / scale < tol
        # the two forms agree to the same order
        assert np.abs(lazy - norm).max() / scale < tol


def test_lazy_rows_are_pivot_multiples_midway():
    """After step k every finished pivot row is d_k times its normalised counterpart."""
    rng = np.random.default_rng(3)
    A = spd(rng, cond=1e3)
    n = 12
    Rl, Rn = A.copy(), A.copy()
    dk = np.zeros(n)
    for k in range(6):
        for R, lazy in ((Rl, True), (Rn, False)):
            d = R[k, k]
            if lazy:
                dk[k] = d
            idv = 1.0 / d
            p = R[k].copy()
            a = -R[:, k] * idv
            if lazy:
                a[k] = 0.0
                col = a.copy()
                col[k] = 1.0
                R += np.outer(a, p)
                R[:, k] = col
            else:
                a[k] = idv
                base = R.copy()
                base[k] = 0.0
                R[:] = base + np.outer(a, p)
                R[:, k] = a
    for k in range(6):
        np.testing.assert_allclose(Rl[k], dk[k] * Rn[k], rtol=1e-10, atol=1e-12 * np.abs(Rl).max())
