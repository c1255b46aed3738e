"""GPU parity at the fixture horizons besides 16 / 32 (test_gpu_parity.py): N = 4j <= 32,
48, round 3's N = 5, 6, 10, 13 (rows past N run as copies of stage N-1; odd N
makes the two sweep chains equally long), 33, 36, 40 (global workspace), 57 and 64
(constraint values in the workspace too), and round 4's 49 (13 waves) and 50 (the
first horizon with the constraint values in the workspace): formulation vs the reference fixtures,
the OSQP solve vs the oracle (statuses and iteration counts equal on every
instance, x within X_TOL), the fused path on a synthetic batch, polish on the
certified optimum x* (sessions: test_gpu_session.py).  The engine compiles every
N from 4 to 64; others are refused with an error code."""
import numpy as np
import pytest
from conftest import FIXTURE_HORIZONS as COMPILED

pytestmark = pytest.mark.gpu

FORM_TOL = 1e-13
X_TOL = 1e-9     # golden QPs (a few hundred iterations), relative to max(1, max |x|)
F_TOL = 5e-8     # fused synthetic batches: longer horizons and up to 4000 iterations amplify
                 # rounding (observed 1.5e-9 at N = 20 with identical iteration counts)


@pytest.fixture(scope="module")
def mpcq():
    import mpcq as M
    return M


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert np.array_equal(np.isinf(a), np.isinf(b))
    fa, fb = np.where(np.isinf(a), 0, a), np.where(np.isinf(b), 0, b)
    return float((np.abs(fa - fb) / np.maximum(1.0, np.abs(fb))).max(initial=0))


def test_supported_horizons(mpcq):
    assert mpcq.supported_horizons() == list(range(4, 65))
    with pytest.raises(mpcq.MpcqError):
        mpcq.Engine(3)
    with pytest.raises(mpcq.MpcqError):
        mpcq.Engine(65)


@pytest.mark.parametrize("N", COMPILED)
def test_horizon_parity(mpcq, golden_h, oracle, N):
    g = golden_h[N]
    with mpcq.Engine(N) as e:
        for mode in (0, 1):
            sfx = "" if mode == 0 else "_setup"
            r = e.formulate(g["xref"], g["fsteps"], mode)
            assert (r["status"] == 0).all()
            err = max(_rel(r["Ax"], g["Ax" + sfx]), _rel(r["l"], g["l" + sfx]), _rel(r["u"], g["u" + sfx]))
            assert err <= FORM_TOL, (mode, err)
        r = e.qp_solve(g["Ax"], g["l"], g["u"])
        for b in range(g["Ax"].shape[0]):
            o = oracle.qp_solve(N, g["Ax"][b], g["l"][b], g["u"][b])
            assert r["status"][b] == o["status"], (b, r["status"][b], o["status"])
            assert r["iters"][b] == o["iters"], (b, r["iters"][b], o["iters"])
            # relative to the solution's scale (|x| up to 25 N at fz_max): 1.1e-9 absolute at N = 64
            assert np.abs(r["x"][b] - o["x"]).max() < X_TOL * max(1.0, np.abs(o["x"]).max())
        # fused formulation + solve on a synthetic mixed-gait batch
        s = mpcq.synth.make_batch(96, N, gaits=mpcq.synth.GAITS, seed=100 + N)
        rf = e.solve(s["xref"], s["fsteps"], 0)
        of = oracle.solve_batch(s["xref"], s["fsteps"], 0, nthreads=16)
        assert np.array_equal(rf["status"], of["status"])
        assert np.array_equal(rf["iters"], of["iters"])
        err = np.abs(rf["f0"] - of["f0"]).max()
        print(f"N={N}: fused max|f0 - f0_oracle| {err:.2e}, iters median {np.median(rf['iters'])}")
        assert err < F_TOL
    over = dict(polish=2, polish_rounds=8, polish_refine_iter=10)
    with mpcq.Engine(N, **over) as e:
        r = e.qp_solve(g["Ax"], g["l"], g["u"])
    assert (r["status"] == 1).all() and (r["polish"] == 1).all()
    d = np.abs(r["x"][:, 12 * N:] - g["x_star"][:, 12 * N:]).max()
    print(f"N={N}: polished max|f - f*| {d:.2e}")
    assert d < 1e-8
