"""Drop-in façade of the reference MPC surface over the HIP engine.

Mirrors, name for name, what the reference's control loop touches:

* ``MPC(dt, n_steps, T_gait)``           -- MPC.py:22-82 (one QP per tick) with
  ``run(k, xref, fsteps)`` (MPC.py:460-514) and the attributes consumers read
  (``f_applied``, ``x``, ``x_robot``, ``xref``, ``q_next``, ``v_next``,
  ``q_w``, ``h_ref``, ``P``, ``n_steps``; Logger.py:156,411-418, utils.py:173).
* ``MPC_Wrapper(dt, n_steps, k_mpc, T_gait, multiprocessing=False)``
  -- MPC_Wrapper.py:20-112: ``solve(k, fstep_planner)`` returns 0,
  ``get_latest_result()`` returns ``[0, 0, 8] * 4`` on its first call
  (MPC_Wrapper.py:64-78), ``run_MPC`` is the compatibility alias named in
  BASELINE.json (stale caller test_motionless.py:63), plus the batched
  ``solve_batch(xref[B,12,N+1], fsteps[B,20,13]) -> f0[B,12]``.
* ``MPC_Virtual(mpc_type, dt_mpc, n_steps, k_mpc, T_gait)`` -- MPC_Virtual.py:20-35.

A tick is one fused launch (mpcq_solve_batch): the formulation (MPC.update_ML /
update_NK, or create_* at k == 0) and the OSQP-0.6 solve with the reference's warm
start (MPC.py:403-406) -- no host round trip between them.  ``ML`` / ``NK`` /
``NK_inf`` (MPC.py:151-234; nothing downstream reads them) are formed on first
access from the tick's inputs by a separate formulation launch.  x is
the previous solution shifted by one stage (states: last stage zeroed; forces:
wrapped, as np.roll does), y and rho carry over from the previous solve as the
osqp workspace does.  The dual is carried the way osqp 0.6 carries it
(params.dual_warm = 1, the façade's default): ``update(Ax=...)`` recomputes the
Ruiz scaling but leaves the workspace y in the previous tick's *scaled*
coordinates, and ``warm_start(x=...)`` (MPC.py:419-420) does not touch it; the
engine then reads and returns that scaled y as is.  ``dual_warm=0`` carries the
unscaled dual instead (osqp's explicit ``warm_start(y=...)``).

Errors: the reference crashes on a gait table without a zero-duration
terminator (MPC.py:636 ``next(...)[0]``) or whose durations do not sum to N
(MPC.py:627 shape error); here both raise ``ValueError``.  Like the reference,
``run`` with k > 0 replaces NaN by 0 in the caller's ``fsteps`` (MPC.py:327).
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .engine import Engine, pattern


def _state_weights(p: L.Params) -> np.ndarray:
    return np.array([p.state_weights[i] for i in range(12)])


class MPC:
    """One receding-horizon QP per tick on the HIP engine (MPC.py:22-514)."""

    def __init__(self, dt, n_steps, T_gait, device: int = 0, engine: Engine | None = None, **overrides):
        self.dt = float(dt)
        self.n_steps = int(n_steps)
        self.T_gait = T_gait
        overrides.setdefault("dual_warm", 1)  # osqp's workspace-y carry-over (MPC.py:419-420)
        self.engine = engine if engine is not None else Engine(self.n_steps, device=device, dt=self.dt, **overrides)
        p = self.engine.params
        self.mass = p.mass
        self.gI = np.array([p.gI[i] for i in range(9)]).reshape(3, 3)
        self.mu = p.mu
        N = self.n_steps
        self.xref = np.zeros((12, 1 + N))
        self.x = np.zeros((24 * N,))
        self.q = np.array([[0.0, 0.0, 0.2027682, 0.0, 0.0, 0.0]]).T
        self.q_w = self.q.copy()
        self.v = np.zeros((6, 1))
        self.h_ref = self.q[2, 0]
        self.footholds = np.array([p.footholds[i] for i in range(12)]).reshape(3, 4)
        # P = diag(weights) (MPC.py:236-288), as a CSC matrix like the reference's
        import scipy.sparse as sp
        diag = np.concatenate([np.tile(_state_weights(p), N), np.full(12 * N, p.force_weight)])
        self.P = sp.diags(diag).tocsc()
        self.Q = np.zeros((24 * N,))
        self._indptr, self._indices = pattern(N)
        self._form = None      # (xref, fsteps, mode) of the last tick, for ML / NK on demand
        self._form_cache = None
        self.x_robot = np.zeros((12, N))
        self.f_applied = np.zeros((12,))
        self.q_next = np.zeros((6, 1))
        self.v_next = np.zeros((6, 1))
        self._y = None
        self._rho = None
        self.status = None
        self.iters = None

    def _warm_x(self):
        """MPC.py:403-406: shift states (zero the last stage) and roll forces."""
        n_x = 12 * self.n_steps
        warmx = np.roll(self.x[:n_x], -12).copy()
        warmx[-12:] = 0
        warmf = np.roll(self.x[n_x:], -12).copy()
        return np.hstack((warmx, warmf))

    def run(self, k, xref, fsteps):
        xref = np.asarray(xref, dtype=np.float64)
        if xref.shape != (12, self.n_steps + 1):
            raise ValueError(f"xref must be (12, {self.n_steps + 1}), got {xref.shape}")
        if np.shape(fsteps) != (20, 13):
            raise ValueError(f"fsteps must be (20, 13), got {np.shape(fsteps)}")
        if k > 0:
            self.q[0:6, 0:1] = xref[0:6, 0:1]
            self.v[0:6, 0:1] = xref[6:12, 0:1]
        self.lC = xref[0:3, 0:1]
        self.xref = xref
        self.x0 = xref[:, 0:1]
        mode = L.MODE_SETUP if k == 0 else L.MODE_UPDATE
        # copies: the caller's planner rewrites xref / fsteps in place every tick
        # (FootstepPlanner.py:96-156), and ML / NK / NK_inf are formed from these later
        xr = np.array(xref, dtype=np.float64, copy=True)[None]
        fs = np.array(fsteps, dtype=np.float64, copy=True)[None]
        if k == 0:
            r = self.engine.solve(xr, fs, mode, want_x=True, want_y=True)
        else:
            r = self.engine.solve(xr, fs, mode, warm_x=self._warm_x(), warm_y=self._y, rho=self._rho,
                                  want_x=True, want_y=True)
        if r["status"][0] == L.STATUS_BAD_GAIT:
            raise ValueError("fsteps: gait table needs a zero-duration terminator and durations summing to n_steps")
        self._form, self._form_cache = (xr, fs, mode), None
        if k > 0:
            fsteps[np.isnan(fsteps)] = 0.0  # MPC.py:327, the caller's array is mutated
        self.status = int(r["status"][0])
        self.iters = int(r["iters"][0])
        self.x = r["x"][0]
        self._y = r["y"][0]
        self._rho = float(r["rho"][0])
        self.retrieve_result()
        # world-frame integration (MPC.py:503-510)
        c_yaw, s_yaw = np.cos(self.q_w[5, 0]), np.sin(self.q_w[5, 0])
        R = np.array([[c_yaw, -s_yaw], [s_yaw, c_yaw]])
        self.q_w[0:2, 0:1] += R @ self.q_next[0:2, 0:1]
        self.q_w[2, 0] = self.q_next[2, 0]
        self.q_w[3:5, 0] = self.q_next[3:5, 0]
        self.q_w[5, 0] += self.q_next[5, 0]
        return 0

    def _formulation(self):
        if self._form is None:
            return None
        if self._form_cache is None:
            xr, fs, mode = self._form
            form = self.engine.formulate(xr, fs, mode)
            import scipy.sparse as sp
            n, m = 24 * self.n_steps, 44 * self.n_steps
            self._form_cache = (sp.csc_matrix((form["Ax"][0], self._indices, self._indptr), shape=(m, n)),
                                form["u"][0].reshape(-1, 1), form["l"][0].copy())
        return self._form_cache

    @property
    def ML(self):
        """A of the last tick's QP (MPC.py:151), CSC in the reference's pattern."""
        f = self._formulation()
        return None if f is None else f[0]

    @property
    def NK(self):
        """u of the last tick's QP as a column (MPC.py:192-234)."""
        f = self._formulation()
        return None if f is None else f[1]

    @property
    def NK_inf(self):
        """l of the last tick's QP (MPC.py:226-232, 410)."""
        f = self._formulation()
        return None if f is None else f[2]

    def retrieve_result(self):
        """MPC.py:432-458."""
        N = self.n_steps
        self.x_robot = self.x[:12 * N].reshape((12, N), order="F").copy()
        self.f_applied = self.x[12 * N:12 * N + 12]
        self.x_robot += self.xref[:, 1:]
        self.q_next = self.x_robot[0:6, 0:1]
        self.v_next = self.x_robot[6:12, 0:1]
        return 0


class MPC_Wrapper:
    """MPC_Wrapper.py:20-290 over the HIP engine.

    ``multiprocessing=False``: ``solve`` runs the tick and returns when it is
    done (MPC_Wrapper.py:83-112).  ``multiprocessing=True``: the asynchronous
    contract the reference sketches with a worker process and shared memory
    (MPC_Wrapper.py:116-215, which its ``solve`` currently refuses to run):
    ``solve`` snapshots the planner's xref / fsteps (replacing NaN by 0 in the
    caller's fsteps, as compress_dataIn does, MPC_Wrapper.py:222) and returns at
    once while the tick runs on a worker thread (the HIP call releases the GIL);
    ``get_latest_result`` hands back that tick's forces once (newResult,
    MPC_Wrapper.py:69-74), waiting for it if it is still running, and raises the
    reference's ValueError when no tick was submitted since the last result."""

    def __init__(self, dt, n_steps, k_mpc, T_gait, multiprocessing=False, device: int = 0,
                 engine: Engine | None = None, **overrides):
        self.f_applied = np.zeros((12,))
        self.not_first_iter = False
        self.k_mpc = k_mpc
        self.multiprocessing = multiprocessing
        self._mpc = MPC(dt, n_steps, T_gait, device=device, engine=engine, **overrides)
        self._pool = None
        self._pending = None
        if multiprocessing:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="mpcq-async")

    @property
    def mpc(self):
        """The MPC object whose attributes Logger / utils read (f_applied, x, x_robot,
        q_w, ...): a tick still running on the worker is waited for first (without
        consuming its result), so readers never see a half-updated object."""
        self._settle()
        return self._mpc

    def _settle(self):
        fut = self._pending
        if fut is not None and not fut.done():
            from concurrent.futures import wait
            wait([fut])

    def solve(self, k, fstep_planner):
        if self.multiprocessing:
            self.run_MPC_asynchronous(k, fstep_planner)
        else:
            self.run_MPC_synchronous(k, fstep_planner)
        return 0

    def run_MPC_asynchronous(self, k, fstep_planner):
        fs = fstep_planner.fsteps
        fs[np.isnan(fs)] = 0.0  # MPC_Wrapper.py:222
        xref, fsteps = np.array(fstep_planner.xref, copy=True), np.array(fs, copy=True)

        mpc = self._mpc

        def job():
            mpc.run(k / self.k_mpc, xref, fsteps)
            return mpc.f_applied.copy()

        self._pending = self._pool.submit(job)
        return 0

    def close(self):
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None

    def run_MPC_synchronous(self, k, fstep_planner):
        self.mpc.run(k / self.k_mpc, fstep_planner.xref, fstep_planner.fsteps)
        self.f_applied = self.mpc.f_applied

    def run_MPC(self, *args):
        """Compatibility alias (BASELINE.json's name).  Accepts ``(k, fstep_planner)`` or the stale
        ``(dt, n_steps, k, T_gait, T_gait/2, joystick, fstep_planner, interface)`` of test_motionless.py:63."""
        if len(args) == 2:
            k, planner = args
        elif len(args) == 8:
            k, planner = args[2], args[6]
        else:
            raise TypeError("run_MPC(k, fstep_planner) or run_MPC(dt, n_steps, k, T_gait, T_gait/2, joystick, "
                            "fstep_planner, interface)")
        return self.solve(k, planner)

    def get_latest_result(self):
        if self.not_first_iter:
            if self.multiprocessing:
                if self._pending is None:
                    raise ValueError("Error: something went wrong with the MPC, result not available.")
                fut, self._pending = self._pending, None
                self.f_applied = fut.result()
                return self.f_applied
            return self.mpc.f_applied
        self.not_first_iter = True
        return np.array([0.0, 0.0, 8.0] * 4)

    def solve_batch(self, xref, fsteps, mode: int = L.MODE_UPDATE, want_x: bool = False):
        """Batched hot path: B independent ticks (cold-started OSQP solves) -> f0 (B, 12).
        Returns (f0, info) with info = dict(status, iters, x)."""
        r = self.mpc.engine.solve(xref, fsteps, mode, want_x=want_x)  # after any pending tick
        return r["f0"], dict(status=r["status"], iters=r["iters"], x=r["x"])


class MPC_Virtual:
    """MPC_Virtual.py:20-35: solve / get_latest_result forwarded to the wrapper."""

    def __init__(self, mpc_type, dt_mpc, n_steps, k_mpc, T_gait, device: int = 0, engine: Engine | None = None):
        if not mpc_type:
            raise ValueError("only mpc_type=True (the OSQP MPC of MPC.py) exists in the reference")
        self.solver = MPC_Wrapper(dt_mpc, n_steps, k_mpc, T_gait, multiprocessing=False, device=device,
                                  engine=engine)
        self.solve = self.solver.solve
        self.get_latest_result = self.solver.get_latest_result
