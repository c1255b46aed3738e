"""Closed-loop sessions: B robots whose whole per-tick MPC state stays in HBM.

``Session(engine, batch)`` wraps ``mpcq_session_*`` (include/mpcq.h).  A tick
is the reference's once-per-tick sequence for every robot —
FootstepPlanner.update_fsteps + getRefStates (processing.py:80-131), MPC.run
(MPC.py:460-514) with osqp's warm start carried over (shifted x, y, rho;
MPC.py:403-406), retrieve_result, the world pose q_w and the Logger's cost
components (Logger.py:406-418) — as three launches on the engine's stream.

Passing ``state=None`` / ``l_feet=None`` runs the virtual robot: the next
state is the previous tick's prediction x_robot[:, 0] re-expressed in the new
local frame (processing.py:33-38 is the reference's precedent).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .engine import Engine


def _shapes(B, N):
    return {
        L.SV_F0: ((B, 12), np.float64), L.SV_X: ((B, 24 * N), np.float64),
        L.SV_X_ROBOT: ((B, 12, N), np.float64), L.SV_Q_W: ((B, 6), np.float64),
        L.SV_COST: ((B, 13), np.float64), L.SV_XREF: ((B, 12, N + 1), np.float64),
        L.SV_FSTEPS: ((B, 20, 13), np.float64), L.SV_GAIT: ((B, 20, 5), np.float64),
        L.SV_STATUS: ((B,), np.int32), L.SV_ITERS: ((B,), np.int32), L.SV_RHO: ((B,), np.float64),
        L.SV_Y: ((B, 44 * N), np.float64), L.SV_STATE: ((B, 12), np.float64),
        L.SV_L_FEET: ((B, 3, 4), np.float64), L.SV_ROT_FLAG: ((B,), np.int32), L.SV_H_ROT: ((B,), np.float64),
        L.SV_ORDER: ((B,), np.int32),
    }


class Session:
    """B robots in closed loop on one engine (device, horizon)."""

    def __init__(self, engine: Engine, batch: int, gait0=None, planner_params: L.PlannerParams | None = None):
        self.engine = engine
        self.batch = int(batch)
        self.n_steps = engine.n_steps
        self.planner_params = planner_params or L.default_planner_params(dt=engine.params.dt)
        self._shapes = _shapes(self.batch, self.n_steps)
        g = None
        if gait0 is not None:
            g = np.ascontiguousarray(np.broadcast_to(np.asarray(gait0, np.float64), (self.batch, 20, 5)))
        h = C.c_void_p()
        self.engine._call("mpcq_session_create", engine._h, self.batch, C.byref(self.planner_params),
                                            None if g is None else C.c_void_p(g.ctypes.data), C.byref(h))
        self._h = h
        self.k = 0

    def close(self):
        if getattr(self, "_h", None):
            L.lib().mpcq_session_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _in(self, a, shape, dtype=np.float64):
        if a is None:
            return None
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(a, dtype), shape))
        return a

    def tick(self, v_ref, state=None, l_feet=None, reduced=None, k: int | None = None):
        """One control tick for every robot (host arrays); returns f_applied (B, 12)."""
        B = self.batch
        k = self.k if k is None else int(k)
        vr = self._in(v_ref, (B, 6))
        st = self._in(state, (B, 12))
        lf = self._in(l_feet, (B, 3, 4))
        rd = self._in(reduced, (B,), np.int32)
        p = lambda a: None if a is None else C.c_void_p(a.ctypes.data)  # noqa: E731
        self.engine._call("mpcq_session_tick", self._h, k, p(st), p(lf), p(vr), p(rd), 0)
        self.k = k + 1
        return self.read(L.SV_F0)

    def tick_device(self, v_ref_ptr: int, state_ptr: int = 0, l_feet_ptr: int = 0, reduced_ptr: int = 0,
                    k: int | None = None, asynchronous: bool = True):
        """One tick on device-resident inputs (pointers on the engine's device)."""
        k = self.k if k is None else int(k)
        v = lambda q: C.c_void_p(q) if q else None  # noqa: E731
        flags = L.FLAG_DEVICE_PTRS | (L.FLAG_ASYNC if asynchronous else 0)
        self.engine._call("mpcq_session_tick", self._h, k, v(state_ptr), v(l_feet_ptr), v(v_ref_ptr), v(reduced_ptr),
                                          flags)
        self.k = k + 1

    def read(self, what: int):
        shape, dt = self._shapes[what]
        out = np.empty(shape, dt)
        self.engine._call("mpcq_session_read", self._h, what, C.c_void_p(out.ctypes.data), 0)
        return out

    def write(self, what: int, value):
        shape, dt = self._shapes[what]
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(value, dt), shape))
        self.engine._call("mpcq_session_write", self._h, what, C.c_void_p(a.ctypes.data), 0)

    def device_ptr(self, what: int) -> int:
        out = C.c_void_p()
        self.engine._call("mpcq_session_device_ptr", self._h, what, C.byref(out))
        return int(out.value or 0)
