"""CPU: pin the oracle (oracle/mpcq_oracle.c) to the reference-generated fixtures.

The fixtures (tests/golden/gen_golden.py) hold the QP data the unmodified
reference MPC.py hands to OSQP and the KKT-certified optimum x*.  These tests
run without a GPU.
"""
import numpy as np
import pytest

FORM_TOL = 1e-14  # formulation: float64 restatement, ulp-level differences only


def _close(a, b, tol):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape
    assert np.array_equal(np.isinf(a), np.isinf(b))
    fa = np.where(np.isinf(a), 0.0, a)
    fb = np.where(np.isinf(b), 0.0, b)
    err = np.abs(fa - fb) / np.maximum(1.0, np.abs(fb))
    return float(err.max(initial=0.0))


@pytest.mark.parametrize("N", [16, 32])
def test_pattern_matches_reference(oracle, N, golden16, golden32):
    g = golden16 if N == 16 else golden32
    indptr, indices = oracle.pattern(N)
    assert np.array_equal(indptr, g["indptr"])
    assert np.array_equal(indices, g["indices"])
    assert g["indices"].size == 126 * N - 18


def test_default_params_match_reference_cost(oracle, golden16):
    p = oracle.default_params()
    N = 16
    Pd = np.concatenate([np.tile(np.array(p.state_weights), N), np.full(12 * N, p.force_weight)])
    assert np.array_equal(Pd, golden16["P"])


@pytest.mark.parametrize("N", [16, 32])
@pytest.mark.parametrize("mode", [0, 1])
def test_formulation_matches_reference(oracle, N, mode, golden16, golden32):
    g = golden16 if N == 16 else golden32
    sfx = "" if mode == 0 else "_setup"
    worst = 0.0
    for b in range(g["xref"].shape[0]):
        Ax, l, u = oracle.formulate(g["xref"][b], g["fsteps"][b], mode)
        worst = max(worst, _close(Ax, g["Ax" + sfx][b], FORM_TOL), _close(l, g["l" + sfx][b], FORM_TOL),
                    _close(u, g["u" + sfx][b], FORM_TOL))
    assert worst <= FORM_TOL, worst


def test_bad_gaits_rejected_like_reference(oracle, golden16):
    # the reference raises (TypeError / ValueError) on all three malformed tables
    assert all(len(s) > 0 for s in golden16["bad_raises"])
    for f in golden16["bad_fsteps"]:
        with pytest.raises(ValueError):
            oracle.formulate(golden16["bad_xref"], f, 0)


def test_golden_optimum_is_certified(golden16, golden32):
    for g in (golden16, golden32):
        assert g["kkt"].max() < 1e-12  # primal, stationarity, sign, complementarity


@pytest.mark.parametrize("N", [16, 32])
def test_oracle_polish_reaches_optimum(oracle, N, golden16, golden32):
    g = golden16 if N == 16 else golden32
    p = oracle.default_params(polish=2, polish_rounds=8, polish_refine_iter=10)
    worst = 0.0
    for b in range(g["xref"].shape[0]):
        r = oracle.qp_solve(N, g["Ax"][b], g["l"][b], g["u"][b], params=p)
        assert r["status"] == 1
        worst = max(worst, np.abs(r["x"][12 * N:] - g["x_star"][b][12 * N:]).max())
    assert worst < 1e-8, worst


def test_oracle_osqp_path_characterisation(oracle, golden16):
    """OSQP-faithful ADMM (polish off, eps 1e-7): status solved, forces within
    the band that OSQP itself leaves around x* on these QPs (a few 1e-3 worst
    case, ~2e-4 median: the force weight 1e-5 makes force space nearly flat)."""
    N = 16
    errs = []
    for b in range(0, golden16["xref"].shape[0], 3):
        r = oracle.qp_solve(N, golden16["Ax"][b], golden16["l"][b], golden16["u"][b])
        assert r["status"] in (1, 2)
        errs.append(np.abs(r["x"][12 * N:12 * N + 12] - golden16["x_star"][b][12 * N:12 * N + 12]).max())
    assert np.median(errs) < 2e-3
    assert max(errs) < 5e-2


def test_oracle_batch_matches_single(oracle, golden16):
    N = 16
    xr, fs = golden16["xref"][:6], golden16["fsteps"][:6]
    rb = oracle.solve_batch(xr, fs, 0, nthreads=2)
    for b in range(6):
        Ax, l, u = oracle.formulate(xr[b], fs[b], 0)
        r = oracle.qp_solve(N, Ax, l, u)
        assert rb["status"][b] == r["status"]
        assert np.array_equal(rb["f0"][b], r["x"][12 * N:12 * N + 12])
