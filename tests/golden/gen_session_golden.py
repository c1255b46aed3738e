"""Generate tests/golden/session_golden.npz (run in the build container only).

    python tests/golden/gen_session_golden.py

Pins what the reference does with a QP solution between two solves — the
parts of a closed-loop tick that are neither the planner nor the solver:

* MPC.retrieve_result (MPC.py:432-458): x_robot, f_applied, q_next, v_next;
* the world-pose integration of MPC.run (MPC.py:503-510): q_w;
* the warm start of the next tick (MPC.py:403-406): the ``initx`` handed to
  osqp's warm_start;
* Logger.log_cost_function (Logger.py:406-418): the 13 cost components.

Drives the UNMODIFIED reference MPC.py and Logger.py with inputs from the
unmodified FootstepPlanner.py (as processing.py:81-131 does).  osqp is absent,
so an in-process stand-in records what MPC.call_solver hands it and returns a
prescribed solution x (seeded random, of the magnitude of real solutions);
the outputs above are then pure functions of (x, xref, q_w) computed by the
reference code.  Other shims: ``np.int = int``, empty ``pybullet``, a
``utils`` module with getSkew (utils.py:179-185).

Only data leaves this script: inputs and expected outputs.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden  # noqa: E402
import gen_planner_golden  # noqa: E402

T_TICKS = 6


class _OsqpScripted(gen_golden._OsqpRecorder):
    """Records the calls; solve() returns the next prescribed x."""

    queue = []

    def solve(self):
        return types.SimpleNamespace(x=_OsqpScripted.queue.pop(0))


def main():
    MPCmod = gen_golden.import_reference_mpc()
    sys.modules["osqp"].OSQP = _OsqpScripted
    MPCmod.osqp.OSQP = _OsqpScripted
    FP = gen_planner_golden.import_reference_planner()
    import Logger  # noqa: E402  (the unmodified reference file; matplotlib is importable here)

    out = {}
    for N, n_periods in ((16, 1), (32, 2)):
        rec = {k: [] for k in ("xref", "fsteps", "x", "x_robot", "f_applied", "q_next", "v_next", "q_w",
                               "initx", "cost")}
        for scen in range(2):
            rng = np.random.default_rng(900 + 10 * N + scen)
            pl = FP.FootstepPlanner(0.02, n_periods)
            mpc = MPCmod.MPC(0.02, N, 0.32)
            log = Logger.Logger(T_TICKS, 0.02, 0.02, 1, n_periods)
            wrapper = types.SimpleNamespace(solver=types.SimpleNamespace(mpc=mpc))
            for j in range(T_TICKS):
                lC, abg, lV, lW, l_feet, v_ref, reduced = gen_planner_golden.draw_inputs(rng, j)
                v_cur = np.vstack((lV, lW))
                if j == 0:
                    pl.update_fsteps(0, l_feet, v_cur, v_ref, lC[2, 0], None, None, reduced)
                pl.update_fsteps(j + 1, l_feet, v_cur, v_ref, lC[2, 0], None, None, reduced)
                pl.getRefStates(float(j), pl.T_gait, lC, abg, lV, lW, v_ref, h_ref=0.2027682)
                # a solution-sized x: states ~ 1e-2, forces ~ 1-10 N
                x = np.concatenate([rng.normal(0, 0.01, 12 * N), rng.normal(2, 3, 12 * N)])
                _OsqpScripted.queue.append(x)
                xref, fsteps = pl.xref.copy(), pl.fsteps.copy()
                mpc.run(j, pl.xref.copy(), pl.fsteps.copy())
                ws = [c for c in mpc.prob.calls if c[0] == "warm_start"]
                initx = ws[-1][1]["x"] if (j > 0 and ws) else np.full(24 * N, np.nan)
                log.log_cost_function(j, wrapper)
                for key, v in (("xref", xref), ("fsteps", fsteps), ("x", x), ("x_robot", mpc.x_robot),
                               ("f_applied", mpc.f_applied), ("q_next", mpc.q_next.ravel()),
                               ("v_next", mpc.v_next.ravel()), ("q_w", mpc.q_w.ravel()), ("initx", initx),
                               ("cost", log.cost_components[:, j])):
                    rec[key].append(np.array(v, copy=True))
        for key, v in rec.items():
            out[f"n{N}_{key}"] = np.stack(v).reshape((2, T_TICKS) + np.shape(v[0]))
    path = os.path.join(HERE, "session_golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
