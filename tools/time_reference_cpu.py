"""Time the reference's own CPU path, in this container only (the reference does
not travel to the GPU box): the unmodified FootstepPlanner tick, MPC.py's
formulation (MPC.run with the osqp stand-in of tests/golden, i.e. everything
but the solve, which cannot run here) and Logger.log_cost_function.

    python tools/time_reference_cpu.py      # writes profiles/r01_reference_cpu.json

Inputs: the seeded synthetic robots of tests/golden/gen_planner_golden.py.
Single thread (numpy/BLAS pinned to one thread).
"""
from __future__ import annotations

import json
import os
import platform
import sys
import time
import types

os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
import gen_golden  # noqa: E402
import gen_planner_golden as gp  # noqa: E402


def main():
    MPCmod = gen_golden.import_reference_mpc()
    FP = gp.import_reference_planner()
    import Logger  # noqa: E402

    class _Solved(gen_golden._OsqpRecorder):
        def solve(self):
            return types.SimpleNamespace(x=np.zeros(self.n))

    MPCmod.osqp.OSQP = _Solved
    out = {"cpu": platform.processor() or platform.machine(), "threads": 1, "note": __doc__.split("\n\n")[0]}
    for N, n_periods in ((16, 1), (32, 2)):
        rng = np.random.default_rng(7)
        pl = FP.FootstepPlanner(0.02, n_periods)
        mpc = MPCmod.MPC(0.02, N, 0.32)
        log = Logger.Logger(200, 0.02, 0.02, 1, n_periods)
        wrapper = types.SimpleNamespace(solver=types.SimpleNamespace(mpc=mpc))
        t_plan, t_form, t_log = [], [], []
        for j in range(60):
            lC, abg, lV, lW, l_feet, v_ref, reduced = gp.draw_inputs(rng, j)
            v_ref[2, 0] = 0.0
            v_cur = np.vstack((lV, lW))
            t0 = time.perf_counter()
            if j == 0:
                pl.update_fsteps(0, l_feet, v_cur, v_ref, lC[2, 0], None, None, False)
            pl.update_fsteps(j + 1, l_feet, v_cur, v_ref, lC[2, 0], None, None, False)
            pl.getRefStates(float(j), pl.T_gait, lC, abg, lV, lW, v_ref, h_ref=0.2027682)
            t1 = time.perf_counter()
            mpc.run(j, pl.xref.copy(), pl.fsteps.copy())
            t2 = time.perf_counter()
            log.log_cost_function(j, wrapper)
            t3 = time.perf_counter()
            if j >= 10:  # after warm-up ticks
                t_plan.append(t1 - t0)
                t_form.append(t2 - t1)
                t_log.append(t3 - t2)
        out[f"N{N}"] = {
            "planner_tick_ms": 1e3 * float(np.median(t_plan)),
            "mpc_formulation_tick_ms": 1e3 * float(np.median(t_form)),
            "logger_cost_ms": 1e3 * float(np.median(t_log)),
            "ticks": len(t_plan),
        }
        print(N, out[f"N{N}"], flush=True)
    path = os.path.join(REPO, "profiles", "r01_reference_cpu.json")
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
