"""CPU: OSQP 0.6's infeasibility detection and l > u rejection in the oracle,
and the dual_warm semantics.

MPC.py's QPs are always feasible (f = 0 with the dynamics roll-out satisfies
every row) and bounded (q = 0, P > 0), so statuses -3 / -4 only come from
hand-made data: a swing force held at 0 by its swing row while its friction
row asks fz >= 10 (primal infeasible).  osqp rejects l > u before solving
(validate_data / osqp_update_bounds; the python wrapper raises): per instance
that is MPCQ_STATUS_BAD_BOUNDS here.  Parity of these paths against the osqp
library is unpinned (osqp is absent); the GPU must equal this
restatement (tests/test_gpu_parity.py)."""
import numpy as np
import pytest

N = 16


def infeasible_instance(g, b):
    """Golden instance b with fz >= 10 N demanded of a foot its swing row holds at 0."""
    Ax, l, u = g["Ax"][b].copy(), g["l"][b].copy(), g["u"][b].copy()
    fs = g["fsteps"][b]
    q = [f for f in range(4) if np.isnan(fs[0, 1 + 3 * f])]
    if not q:
        return None
    u[24 * N + 5 * q[0] + 4] = -10.0  # row 5 of C: -fz <= u  ->  fz >= 10 at stage 0
    return Ax, l, u


def test_primal_infeasible_detected(oracle, golden16):
    seen = 0
    for b in range(0, 50, 5):
        inst = infeasible_instance(golden16, b)
        if inst is None:
            continue
        r = oracle.qp_solve(N, *inst)
        assert r["status"] == -3, (b, r["status"])
        assert r["iters"] < 4000 and r["iters"] % 25 == 0  # found at a termination check
        assert np.isnan(r["x"]).all() and np.isnan(r["y"]).all()  # osqp store_solution
        seen += 1
    assert seen >= 5


def test_feasible_instances_never_flagged(oracle, golden16, golden32):
    for g, n_ in ((golden16, 16), (golden32, 32)):
        for b in range(g["Ax"].shape[0]):
            assert oracle.qp_solve(n_, g["Ax"][b], g["l"][b], g["u"][b])["status"] in (1, 2)


def test_infeasible_before_max_iter(oracle, golden16):
    """max_iter below the detection point: MAX_ITER_REACHED, then -3 once a
    (final) check sees the certificate."""
    Ax, l, u = infeasible_instance(golden16, 0)
    st = [oracle.qp_solve(N, Ax, l, u, params=oracle.default_params(max_iter=mi))["status"]
          for mi in (30, 60, 100, 101, 110, 4000)]
    assert st == [-2, -2, -2, -3, -3, -3]


def test_l_greater_than_u_rejected(oracle, golden16):
    Ax, l, u = golden16["Ax"][0], golden16["l"][0].copy(), golden16["u"][0]
    l[24 * N + 3] = 1.0  # friction row: u = 0 < l
    r = oracle.qp_solve(N, Ax, l, u)
    assert r["status"] == -13 and np.isnan(r["x"]).all()


def test_dual_warm_semantics(oracle, golden16):
    """dual_warm = 1 returns / takes the solver's scaled y.  Cold, both modes run
    the same iterations; warm-started on the SAME data (same scaling) the two
    carry-overs coincide; on the next tick's data they differ (osqp's scaled y
    is not re-scaled by update(Ax=))."""
    g = golden16
    p0, p1 = oracle.default_params(), oracle.default_params(dual_warm=1)
    Ax, l, u = g["Ax"][3], g["l"][3], g["u"][3]
    r0 = oracle.qp_solve(N, Ax, l, u, params=p0)
    r1 = oracle.qp_solve(N, Ax, l, u, params=p1)
    assert r0["iters"] == r1["iters"] and np.array_equal(r0["x"], r1["x"])
    assert not np.allclose(r0["y"], r1["y"])  # unscaled vs scaled coordinates
    w0 = oracle.qp_solve(N, Ax, l, u, params=p0, warm_x=r0["x"], warm_y=r0["y"], rho=r0["rho"])
    w1 = oracle.qp_solve(N, Ax, l, u, params=p1, warm_x=r1["x"], warm_y=r1["y"], rho=r1["rho"])
    assert w0["iters"] == w1["iters"]
    assert np.abs(w0["x"] - w1["x"]).max() < 1e-12
    Ax2, l2, u2 = g["Ax"][4], g["l"][4], g["u"][4]
    v0 = oracle.qp_solve(N, Ax2, l2, u2, params=p0, warm_x=r0["x"], warm_y=r0["y"], rho=r0["rho"])
    v1 = oracle.qp_solve(N, Ax2, l2, u2, params=p1, warm_x=r1["x"], warm_y=r1["y"], rho=r1["rho"])
    assert v0["status"] == v1["status"] == 1
    assert np.abs(v0["x"] - v1["x"]).max() > 0.0


@pytest.mark.parametrize("dual_warm", [0, 1])
def test_session_oracle_dual_warm(oracle, dual_warm):
    """The composed closed loop runs in both modes (the GPU sessions are checked
    against it tick by tick in tests/test_gpu_session.py)."""
    from mpcq import synth
    s = oracle.Session(N, synth.gait_table("trot", N), params=oracle.default_params(dual_warm=dual_warm))
    for k in range(4):
        s.tick(k, np.array([0.3, 0.0, 0.0, 0.0, 0.0, 0.2]))
        assert s.status in (1, 2)
