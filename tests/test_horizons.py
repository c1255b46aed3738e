"""CPU: the oracle at the fixture horizons (N = 4j <= 32, N = 48 = n_periods 3;
round 3: N = 5, 6, 10, 13, 33, 36, 40, 57 and 64 = n_periods 4), pinned to
fixtures captured from the unmodified reference MPC.py (tests/golden/gen_golden.py
horizons / horizons_r3): the CSC pattern, the
A / l / u handed to OSQP in both modes, and the polished solve on the certified
optimum x*.  The reference takes any n_steps (MPC.py:22-26; FootstepPlanner.py:55
n_steps = n_periods T_gait / dt)."""
import numpy as np
import pytest
from conftest import FIXTURE_HORIZONS as HORIZONS

FORM_TOL = 1e-14


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    assert np.array_equal(np.isinf(a), np.isinf(b))
    fa, fb = np.where(np.isinf(a), 0.0, a), np.where(np.isinf(b), 0.0, b)
    return float((np.abs(fa - fb) / np.maximum(1.0, np.abs(fb))).max(initial=0.0))


def test_fixture_horizons(golden_h):
    assert tuple(sorted(golden_h)) == HORIZONS
    for N, g in golden_h.items():
        assert g["Ax"].shape[1] == 126 * N - 18
        assert g["l"].shape[1] == 44 * N
        assert g["kkt"].max() < 1e-12  # x* certified by its KKT residuals


@pytest.mark.parametrize("N", HORIZONS)
def test_pattern(oracle, golden_h, N):
    indptr, indices = oracle.pattern(N)
    assert np.array_equal(indptr, golden_h[N]["indptr"])
    assert np.array_equal(indices, golden_h[N]["indices"])


@pytest.mark.parametrize("N", HORIZONS)
@pytest.mark.parametrize("mode", [0, 1])
def test_formulation(oracle, golden_h, N, mode):
    g = golden_h[N]
    sfx = "" if mode == 0 else "_setup"
    worst = 0.0
    for b in range(g["xref"].shape[0]):
        Ax, l, u = oracle.formulate(g["xref"][b], g["fsteps"][b], mode)
        worst = max(worst, _rel(Ax, g["Ax" + sfx][b]), _rel(l, g["l" + sfx][b]), _rel(u, g["u" + sfx][b]))
    assert worst <= FORM_TOL, worst


@pytest.mark.parametrize("N", HORIZONS)
def test_polish_reaches_optimum(oracle, golden_h, N):
    g = golden_h[N]
    p = oracle.default_params(polish=2, polish_rounds=8, polish_refine_iter=10)
    worst = 0.0
    for b in range(g["xref"].shape[0]):
        r = oracle.qp_solve(N, g["Ax"][b], g["l"][b], g["u"][b], params=p)
        assert r["status"] == 1
        worst = max(worst, np.abs(r["x"][12 * N:] - g["x_star"][b][12 * N:]).max())
    assert worst < 1e-8, worst


@pytest.mark.parametrize("N", HORIZONS)
def test_bad_gaits_rejected_like_reference(oracle, golden_h, N):
    g = golden_h[N]
    assert all(len(s) > 0 for s in g["bad_raises"])
    for f in g["bad_fsteps"]:
        with pytest.raises(ValueError):
            oracle.formulate(g["bad_xref"], f, 0)
