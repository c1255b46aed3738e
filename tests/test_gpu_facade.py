"""GPU: the drop-in façade (MPC_Wrapper over the HIP engine) over a short
closed loop -- setup tick then warm-started update ticks carrying x, y and rho
-- against the same façade driven by the oracle (tests/facade_util.py)."""
import numpy as np
import pytest

from facade_util import OracleEngine, Planner

pytestmark = pytest.mark.gpu
TOL = 1e-8  # |x_gpu - x_oracle| per tick (same iterations; fp64 rounding only)


def test_closed_loop_matches_oracle(golden16, oracle):
    from mpcq.wrapper import MPC_Wrapper
    w_gpu = MPC_Wrapper(0.02, 16, 20, 0.32, device=0)
    w_ora = MPC_Wrapper(0.02, 16, 20, 0.32, engine=OracleEngine(oracle))
    assert w_gpu.get_latest_result().tolist() == [0.0, 0.0, 8.0] * 4
    for tick in range(5):
        b = tick % 3
        for w in (w_gpu, w_ora):
            w.solve(20 * tick, Planner(golden16["xref"][b], golden16["fsteps"][b]))
        a, o = w_gpu.mpc, w_ora.mpc
        assert a.status == o.status == 1, (tick, a.status, o.status)
        assert a.iters == o.iters, (tick, a.iters, o.iters)
        assert np.abs(a.x - o.x).max() < TOL, tick
        assert abs(a._rho - o._rho) <= 1e-6 * o._rho  # rho = f(residual ratio): rounding-sensitive
        assert np.allclose(a.q_w, o.q_w, atol=TOL)


def test_solve_batch(golden16, oracle):
    from mpcq.wrapper import MPC_Wrapper
    w = MPC_Wrapper(0.02, 16, 20, 0.32, device=0)
    f0, info = w.solve_batch(golden16["xref"][:8], golden16["fsteps"][:8])
    ref = oracle.solve_batch(golden16["xref"][:8], golden16["fsteps"][:8], 0, nthreads=4)
    assert np.array_equal(info["status"], ref["status"])
    assert np.abs(f0 - ref["f0"]).max() < 1e-6
