"""CPU: the session epilogue restatement (oracle/session_oracle.c) against
fixtures captured from the unmodified MPC.py / Logger.py
(tests/golden/gen_session_golden.py): x_robot, the world pose q_w, the next
tick's warm start and the Logger's cost components, bit for bit; and the
composed one-robot closed loop of the oracle (oracle.Session) on a few ticks."""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "session_golden.npz")


@pytest.mark.parametrize("N", [16, 32])
def test_retrieve_oracle_bit_exact(N):
    G = np.load(GOLD)
    S, T = G[f"n{N}_x"].shape[:2]
    for s in range(S):
        qw = np.array([0.0, 0.0, 0.2027682, 0.0, 0.0, 0.0])  # MPC.py:53-56
        prev_warm = None
        for j in range(T):
            o = O.retrieve(N, G[f"n{N}_x"][s, j], G[f"n{N}_xref"][s, j], G[f"n{N}_fsteps"][s, j],
                           np.zeros((20, 5)), qw)
            qw = o["q_w"]
            assert np.array_equal(o["x_robot"], G[f"n{N}_x_robot"][s, j])
            assert np.array_equal(o["x_robot"][0:6, 0], G[f"n{N}_q_next"][s, j])
            assert np.array_equal(o["x_robot"][6:12, 0], G[f"n{N}_v_next"][s, j])
            assert np.array_equal(qw, G[f"n{N}_q_w"][s, j])
            assert np.array_equal(o["cost"], G[f"n{N}_cost"][s, j])
            if j > 0:  # warm_start(x=initx) of tick j is built from tick j-1's solution
                assert np.array_equal(prev_warm, G[f"n{N}_initx"][s, j])
            prev_warm = o["warm_x"]


def test_oracle_session_closed_loop():
    """The virtual robot walks (trot, 1 m/s): every tick solves, the warm start
    (shifted x, y, rho) makes later ticks cheaper than the first."""
    from mpcq import synth
    s = O.Session(16, synth.gait_table("trot", 16))
    v_ref = np.array([0.5, 0.0, 0.0, 0.0, 0.0, 0.2])
    iters = []
    for k in range(6):
        assert s.tick(k, v_ref) == 1
        iters.append(s.iters)
        assert np.isfinite(s.f0).all() and np.isfinite(s.state).all()
    assert np.median(iters[1:]) < iters[0], iters
    assert s.q_w[0] > 0.0  # it moved forward in the world
