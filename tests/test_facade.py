"""CPU: host logic of the drop-in façade (mpcq/wrapper.py) with the oracle
standing in for the device engine (tests/facade_util.py)."""
import numpy as np
import pytest

from facade_util import OracleEngine, Planner


@pytest.fixture()
def wrapper(oracle):
    from mpcq.wrapper import MPC_Wrapper
    return MPC_Wrapper(0.02, 16, 20, 0.32, engine=OracleEngine(oracle))


def test_first_result_is_default_forces(wrapper, golden16):
    w = wrapper
    assert np.array_equal(w.get_latest_result(), np.array([0.0, 0.0, 8.0] * 4))
    pl = Planner(golden16["xref"][0], golden16["fsteps"][0])
    assert w.solve(0, pl) == 0
    f = w.get_latest_result()
    assert f.shape == (12,)
    assert np.array_equal(f, w.mpc.x[192:204])


def test_tick_sequence_and_attributes(wrapper, golden16, oracle):
    w, N = wrapper, 16
    xr, fs = golden16["xref"][0], golden16["fsteps"][0]
    pl = Planner(xr, fs)
    w.solve(0, pl)                      # k = 0: setup formulation (default footholds), cold start
    x0 = w.mpc.x.copy()
    assert np.isnan(pl.fsteps).any()    # not mutated at k == 0 (update_ML is not called)
    w.solve(20, pl)                     # k / k_mpc = 1: update formulation, warm start
    assert not np.isnan(pl.fsteps).any()  # MPC.py:327 mutates the caller's fsteps
    eng = w.mpc.engine
    assert eng.calls[0]["warm_x"] is None and eng.calls[0]["rho"] is None
    wx = eng.calls[1]["warm_x"]
    # MPC.py:403-406: states shifted by one stage with the last zeroed; forces rolled (wrapping)
    assert np.array_equal(wx[:12 * N - 12], x0[12:12 * N]) and not wx[12 * N - 12:12 * N].any()
    assert np.array_equal(wx[12 * N:], np.roll(x0[12 * N:], -12))
    assert eng.calls[1]["warm_y"] is not None and eng.calls[1]["rho"] > 0
    m = w.mpc
    assert m.x_robot.shape == (12, N) and m.q_next.shape == (6, 1) and m.v_next.shape == (6, 1)
    assert np.allclose(m.x_robot, m.x[:12 * N].reshape(12, N, order="F") + xr[:, 1:])
    assert m.P.shape == (24 * N, 24 * N) and np.array_equal(m.P.diagonal(), golden16["P"])
    assert m.ML.shape == (44 * N, 24 * N) and m.ML.nnz == 126 * N - 18
    # the same tick straight through the oracle
    Ax, l, u = oracle.formulate(xr, fs, 0)
    r = oracle.qp_solve(N, Ax, l, u, warm_x=wx, warm_y=eng.calls[1]["warm_y"], rho=eng.calls[1]["rho"])
    assert np.array_equal(r["x"], m.x)


def test_formulation_attributes_keep_the_solved_qp(wrapper, golden16, oracle):
    """ML / NK / NK_inf describe the QP run() solved, even after the caller's planner
    rewrites xref / fsteps in place for the next tick (FootstepPlanner.py:96-156)."""
    w, N = wrapper, 16
    pl = Planner(golden16["xref"][0], golden16["fsteps"][0])
    w.solve(0, pl)
    w.solve(20, pl)
    Ax, l, u = oracle.formulate(golden16["xref"][0], np.nan_to_num(golden16["fsteps"][0]), 0)
    pl.xref += 0.05           # the planner's in-place update of the next tick
    pl.fsteps[:, 1:] += 0.01
    m = w.mpc
    assert np.array_equal(m.ML.data, Ax)
    assert np.array_equal(m.NK.ravel(), u)
    assert np.array_equal(m.NK_inf, l)


def test_run_mpc_alias_and_virtual(oracle, golden16):
    from mpcq.wrapper import MPC_Virtual, MPC_Wrapper
    w = MPC_Wrapper(0.02, 16, 20, 0.32, engine=OracleEngine(oracle))
    pl = Planner(golden16["xref"][1], golden16["fsteps"][1])
    assert w.run_MPC(0, pl) == 0
    f_a = w.mpc.f_applied.copy()
    w2 = MPC_Wrapper(0.02, 16, 20, 0.32, engine=OracleEngine(oracle))
    # stale signature of test_motionless.py:63 (dt, n_steps, k, T_gait, T_gait/2, joystick, planner, interface)
    assert w2.run_MPC(0.02, 16, 0, 0.32, 0.16, None, Planner(golden16["xref"][1], golden16["fsteps"][1]), None) == 0
    assert np.array_equal(f_a, w2.mpc.f_applied)
    with pytest.raises(TypeError):
        w.run_MPC(1, 2, 3)
    v = MPC_Virtual(True, 0.02, 16, 20, 0.32, engine=OracleEngine(oracle))
    assert v.solve(0, pl) == 0 and v.get_latest_result().tolist() == [0.0, 0.0, 8.0] * 4
    with pytest.raises(ValueError):
        MPC_Virtual(False, 0.02, 16, 20, 0.32, engine=OracleEngine(oracle))


def test_errors(oracle, golden16):
    from mpcq.wrapper import MPC_Wrapper
    # asynchronous: the tick's error surfaces where its result is collected
    w = MPC_Wrapper(0.02, 16, 20, 0.32, multiprocessing=True, engine=OracleEngine(oracle))
    w.get_latest_result()
    w.solve(0, Planner(golden16["xref"][0], golden16["bad_fsteps"][0]))
    with pytest.raises(ValueError):
        w.get_latest_result()
    w.close()
    w = MPC_Wrapper(0.02, 16, 20, 0.32, engine=OracleEngine(oracle))
    with pytest.raises(ValueError):
        w.solve(0, Planner(golden16["xref"][0], golden16["bad_fsteps"][0]))
    with pytest.raises(ValueError):
        w.solve(0, Planner(golden16["xref"][0][:, :5], golden16["fsteps"][0]))


def test_async_wrapper_contract(oracle, golden16):
    """multiprocessing=True: solve returns at once, get_latest_result hands each
    tick's forces back once (MPC_Wrapper.py:64-78, 116-215)."""
    from mpcq.wrapper import MPC_Wrapper
    w = MPC_Wrapper(0.02, 16, 20, 0.32, multiprocessing=True, engine=OracleEngine(oracle))
    s = MPC_Wrapper(0.02, 16, 20, 0.32, engine=OracleEngine(oracle))
    assert w.get_latest_result().tolist() == [0.0, 0.0, 8.0] * 4
    s.get_latest_result()
    with pytest.raises(ValueError):
        w.get_latest_result()  # nothing submitted
    for tick in range(3):
        pl = Planner(golden16["xref"][tick], golden16["fsteps"][tick])
        pl2 = Planner(golden16["xref"][tick], golden16["fsteps"][tick])
        assert w.solve(20 * tick, pl) == 0
        assert not np.isnan(pl.fsteps).any()  # compress_dataIn's NaN -> 0 (MPC_Wrapper.py:222)
        s.solve(20 * tick, pl2)
        assert np.array_equal(w.get_latest_result(), s.get_latest_result())
        with pytest.raises(ValueError):
            w.get_latest_result()  # consumed
    w.close()


def test_footstep_planner_facade_errors_without_device():
    """The planner façade has no CPU fallback: without a HIP device it raises."""
    import mpcq
    from mpcq.planner import FootstepPlanner
    with pytest.raises(mpcq.MpcqError):
        FootstepPlanner(0.02, 1)
