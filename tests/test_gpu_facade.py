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
    w_ora = MPC_Wrapper(0.02, 16, 20, 0.32, engine=OracleEngine(oracle, dual_warm=1))
    assert w_gpu.mpc.engine.params.dual_warm == 1  # the façade carries osqp's scaled y
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
    assert np.array_equal(info["iters"], ref["iters"])
    assert np.abs(f0 - ref["f0"]).max() < 1e-9  # same algorithm, fp64 rounding only (observed ~1e-12)


def test_footstep_planner_facade_vs_reference_fixtures():
    """The drop-in FootstepPlanner (one robot on the GPU) driven exactly as the
    reference control loop drives the reference class (processing.py:80-131)
    reproduces the captured reference states (tests/golden/planner_golden.npz)."""
    import os
    from mpcq.planner import FootstepPlanner
    G = np.load(os.path.join(os.path.dirname(__file__), "golden", "planner_golden.npz"))
    for N, n_periods in ((16, 1), (32, 2)):
        for s in range(G[f"n{N}_state"].shape[0]):
            pl = FootstepPlanner(0.02, n_periods)
            if str(G[f"n{N}_kind"][s]) != "trot":
                pl.gait = G[f"n{N}_gait0"][s].copy()
            assert np.array_equal(pl.gait, G[f"n{N}_gait0"][s])
            for j in range(6):
                st = G[f"n{N}_state"][s, j]
                lC, abg, lV, lW = st[0:3, None], st[3:6, None], st[6:9, None], st[9:12, None]
                lf, vr, red = G[f"n{N}_l_feet"][s, j], G[f"n{N}_v_ref"][s, j][:, None], bool(G[f"n{N}_reduced"][s, j])
                v_cur = np.vstack((lV, lW))
                if j == 0:
                    pl.update_fsteps(0, lf, v_cur, vr, lC[2, 0], None, None, red)
                pl.update_fsteps(j * 20 + 1, lf, v_cur, vr, lC[2, 0], None, None, red)
                pl.getRefStates(float(j), pl.T_gait, lC, abg, lV, lW, vr, h_ref=0.2027682)
                assert np.array_equal(pl.gait, G[f"n{N}_gait"][s, j]), (N, s, j)
                assert pl.flag_rotation_command == G[f"n{N}_flag"][s, j]
                assert np.array_equal(np.isnan(pl.fsteps), np.isnan(G[f"n{N}_fsteps"][s, j]))
                assert np.nanmax(np.abs(pl.fsteps - G[f"n{N}_fsteps"][s, j])) <= 1e-15
                assert np.abs(pl.xref - G[f"n{N}_xref"][s, j]).max() <= 1e-15
            pl.engine.close()
    bad = FootstepPlanner(0.02, 1)
    bad.gait = G["bad_gait"].copy()
    with pytest.raises(TypeError):
        bad.roll()
    with pytest.raises(IndexError):
        bad.compute_footsteps(np.zeros((3, 4)), np.zeros((6, 1)), np.zeros((6, 1)), 0.2, False)


def test_async_wrapper_matches_sync(golden16):
    """multiprocessing=True on the GPU: the worker-thread tick returns what the
    synchronous wrapper returns."""
    from mpcq.wrapper import MPC_Wrapper
    wa = MPC_Wrapper(0.02, 16, 20, 0.32, multiprocessing=True, device=0)
    ws = MPC_Wrapper(0.02, 16, 20, 0.32, device=0)
    wa.get_latest_result()
    ws.get_latest_result()
    for tick in range(4):
        b = tick % 3
        wa.solve(20 * tick, Planner(golden16["xref"][b], golden16["fsteps"][b]))
        ws.solve(20 * tick, Planner(golden16["xref"][b], golden16["fsteps"][b]))
        assert np.array_equal(wa.get_latest_result(), ws.get_latest_result())
    wa.close()


def test_async_wrapper_shares_engine_safely(golden16):
    """A batched solve and attribute reads while an asynchronous tick is in flight
    on the same context: the context lock serialises the calls, reads wait for the
    tick, and both results equal the ones computed without overlap."""
    from mpcq.wrapper import MPC_Wrapper
    wa = MPC_Wrapper(0.02, 16, 20, 0.32, multiprocessing=True, device=0)
    ws = MPC_Wrapper(0.02, 16, 20, 0.32, device=0)
    wa.get_latest_result()
    ws.get_latest_result()
    xb, fb = golden16["xref"][:32], golden16["fsteps"][:32]
    ref_batch, _ = ws.solve_batch(xb, fb)
    for tick in range(3):
        b = tick % 3
        wa.solve(20 * tick, Planner(golden16["xref"][b], golden16["fsteps"][b]))
        f_batch, _ = wa.solve_batch(xb, fb)          # issued while the tick may still run
        xr = wa.mpc.x_robot.copy()                   # waits for the tick
        ws.solve(20 * tick, Planner(golden16["xref"][b], golden16["fsteps"][b]))
        assert np.array_equal(f_batch, ref_batch)
        assert np.array_equal(wa.get_latest_result(), ws.get_latest_result())
        assert np.array_equal(xr, ws.mpc.x_robot)
    wa.close()
