"""Batched engine: numpy (host) and device-pointer front ends over libmpcq.so.

``Engine(n_steps)`` is the batched counterpart of one ``MPC.MPC`` +
``osqp.OSQP`` pair (MPC.py:22-82): it owns a HIP context on one device.

* ``formulate(xref, fsteps, mode)``  -> A.data / l / u exactly as
  MPC.update_matrices (MPC.py:290-378) or create_matrices (MPC.py:84-234).
* ``qp_solve(Ax, l, u, ...)``        -> osqp update + warm_start + solve
  (MPC.py:419-428) for every instance.
* ``solve(xref, fsteps, mode, ...)`` -> the fused hot path of MPC.run
  (MPC.py:460-514): formulation + solve + f_applied.

Host arrays go through pinned-free staging inside the library; the
``*_device`` variants take raw device pointers (e.g. ``tensor.data_ptr()``)
so callers can keep inputs resident in HBM and time the kernel alone.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np

from . import _lib as L


def dims(n_steps: int):
    return 24 * n_steps, 44 * n_steps, 126 * n_steps - 18


def pattern(n_steps: int):
    n, m, nnz = dims(n_steps)
    indptr = np.zeros(n + 1, np.int32)
    indices = np.zeros(nnz, np.int32)
    L.check(L.lib().mpcq_pattern(n_steps, indptr.ctypes.data_as(C.POINTER(C.c_int32)),
                                 indices.ctypes.data_as(C.POINTER(C.c_int32))))
    return indptr, indices


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _f64(a, shape=None):
    if a is None:
        return None
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None and a.shape != shape:
        raise ValueError(f"expected shape {shape}, got {a.shape}")
    return a


class Engine:
    """One HIP context (device, horizon N, parameters)."""

    def __init__(self, n_steps: int = 16, device: int = 0, params: L.Params | None = None, **overrides):
        self.n_steps = int(n_steps)
        self.device = int(device)
        self.params = params if params is not None else L.default_params()
        for k, v in overrides.items():
            setattr(self.params, k, v)
        self.n, self.m, self.nnz = dims(self.n_steps)
        self.lock = threading.RLock()
        h = C.c_void_p()
        L.check(L.lib().mpcq_create(self.device, self.n_steps, C.byref(self.params), C.byref(h)))
        self._h = h

    def _call(self, name: str, *args):
        """One C-ABI call on this context.  A context is used by one host thread at a
        time (include/mpcq.h): the lock serialises callers that share the Engine
        (the asynchronous MPC_Wrapper's worker and the caller's thread)."""
        with self.lock:
            return L.check(getattr(L.lib(), name)(*args))

    def close(self):
        if getattr(self, "_h", None):
            with self.lock:
                L.lib().mpcq_destroy(self._h)
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

    # ------------------------------------------------------------------ host arrays
    def _batch_inputs(self, xref, fsteps):
        xref = _f64(xref)
        fsteps = _f64(fsteps)
        if xref.ndim == 2:
            xref = xref[None]
        if fsteps.ndim == 2:
            fsteps = fsteps[None]
        B = xref.shape[0]
        if xref.shape != (B, 12, self.n_steps + 1) or fsteps.shape != (B, 20, 13):
            raise ValueError(f"xref must be (B,12,{self.n_steps + 1}) and fsteps (B,20,13); got "
                             f"{xref.shape}, {fsteps.shape}")
        return np.ascontiguousarray(xref), np.ascontiguousarray(fsteps), B

    def formulate(self, xref, fsteps, mode: int = L.MODE_UPDATE):
        xref, fsteps, B = self._batch_inputs(xref, fsteps)
        Ax = np.empty((B, self.nnz))
        l = np.empty((B, self.m))
        u = np.empty((B, self.m))
        st = np.empty(B, np.int32)
        self._call("mpcq_formulate_batch", self._h, B, _p(xref), _p(fsteps), mode, _p(Ax), _p(l), _p(u),
                                             _p(st), 0)
        return dict(Ax=Ax, l=l, u=u, status=st)

    def qp_solve(self, Ax, l, u, warm_x=None, warm_y=None, rho=None, want_y: bool = True):
        Ax = _f64(Ax)
        B = Ax.shape[0] if Ax.ndim == 2 else 1
        Ax = Ax.reshape(B, self.nnz)
        l = _f64(l).reshape(B, self.m)
        u = _f64(u).reshape(B, self.m)
        wx = None if warm_x is None else _f64(warm_x).reshape(B, self.n)
        wy = None if warm_y is None else _f64(warm_y).reshape(B, self.m)
        rho_in = None if rho is None else np.ascontiguousarray(np.broadcast_to(np.asarray(rho, np.float64), (B,)))
        x = np.empty((B, self.n))
        y = np.empty((B, self.m)) if want_y else None
        st = np.empty(B, np.int32)
        it = np.empty(B, np.int32)
        ro = np.empty(B)
        info = np.empty((B, 4), np.int32)
        self._call("mpcq_qp_solve_batch", self._h, B, _p(Ax), _p(l), _p(u), _p(wx), _p(wy), _p(rho_in),
                                            _p(x), _p(y), _p(st), _p(it), _p(ro), _p(info), 0)
        return dict(x=x, y=y, status=st, iters=it, rho=ro, rho_updates=info[:, 0], polish=info[:, 1],
                    polish_rounds=info[:, 2], admm_status=info[:, 3])

    def solve(self, xref, fsteps, mode: int = L.MODE_UPDATE, warm_x=None, warm_y=None, rho=None,
              want_x: bool = True, want_y: bool = False, order_by_class: bool = False):
        """Fused formulation + solve (mpcq_solve_batch): MPC.run's QP for a batch, with
        the osqp workspace of the previous tick (warm_x, warm_y, rho) when given.
        order_by_class: MPCQ_FLAG_ORDER_BY_CLASS (dispatch by the mean iteration count each
        gait class has shown on this engine; results unchanged)."""
        xref, fsteps, B = self._batch_inputs(xref, fsteps)
        wx = None if warm_x is None else _f64(warm_x).reshape(B, self.n)
        wy = None if warm_y is None else _f64(warm_y).reshape(B, self.m)
        rin = None if rho is None else np.ascontiguousarray(np.broadcast_to(np.asarray(rho, np.float64), (B,)))
        f0 = np.empty((B, 12))
        x = np.empty((B, self.n)) if want_x else None
        y = np.empty((B, self.m)) if want_y else None
        rout = np.empty(B)
        st = np.empty(B, np.int32)
        it = np.empty(B, np.int32)
        info = np.empty((B, 4), np.int32)
        self._call("mpcq_solve_batch", self._h, B, _p(xref), _p(fsteps), mode, _p(wx), _p(wy), _p(rin), _p(f0),
                                         _p(x), _p(y), _p(rout), _p(st), _p(it), _p(info),
                   L.FLAG_ORDER_BY_CLASS if order_by_class else 0)
        return dict(f0=f0, x=x, y=y, rho=rout, status=st, iters=it, rho_updates=info[:, 0], polish=info[:, 1],
                    polish_rounds=info[:, 2], admm_status=info[:, 3])

    # ------------------------------------------------------------------ footstep planner
    def plan(self, ops: int, k: int, state, l_feet, v_ref, gait, rot_flag, h_rot, xref, fsteps,
             reduced=None, v_cur=None, h=None, params: L.PlannerParams | None = None):
        """FootstepPlanner.update_fsteps + getRefStates for a batch (mpcq_plan_batch).

        ``gait`` (B,20,5), ``rot_flag`` (B,) int32, ``h_rot`` (B,), ``xref`` (B,12,N+1) and
        ``fsteps`` (B,20,13) are C-contiguous arrays updated in place.  Returns status (B,):
        0, or STATUS_BAD_GAIT where the reference raises (that instance left unchanged)."""
        B = int(np.shape(state)[0])
        N = self.n_steps
        state = _f64(state, (B, 12))
        v_ref = _f64(v_ref, (B, 6))
        l_feet = None if l_feet is None else _f64(l_feet, (B, 3, 4))
        v_cur = None if v_cur is None else _f64(v_cur, (B, 6))
        h = None if h is None else _f64(h, (B,))
        red = None if reduced is None else np.ascontiguousarray(np.broadcast_to(np.asarray(reduced, np.int32), (B,)))
        for name, arr, shp, dt in (("gait", gait, (B, 20, 5), np.float64), ("rot_flag", rot_flag, (B,), np.int32),
                                   ("h_rot", h_rot, (B,), np.float64), ("xref", xref, (B, 12, N + 1), np.float64),
                                   ("fsteps", fsteps, (B, 20, 13), np.float64)):
            if arr is None:
                continue
            if arr.shape != shp or arr.dtype != dt or not arr.flags.c_contiguous:
                raise ValueError(f"{name} must be a C-contiguous {np.dtype(dt).name} array of shape {shp}")
        st = np.empty(B, np.int32)
        pp = params if params is not None else L.default_planner_params(dt=self.params.dt)
        self._call("mpcq_plan_batch", self._h, C.byref(pp), B, ops, int(k), _p(state), _p(v_cur), _p(h),
                                        _p(l_feet), _p(v_ref), _p(red), _p(gait), _p(rot_flag), _p(h_rot),
                                        _p(xref), _p(fsteps), _p(st), 0)
        return st

    def plan_device(self, batch: int, ops: int, k: int, state_ptr: int, l_feet_ptr: int, v_ref_ptr: int,
                    gait_ptr: int, rot_flag_ptr: int, h_rot_ptr: int, xref_ptr: int, fsteps_ptr: int,
                    status_ptr: int = 0, reduced_ptr: int = 0, v_cur_ptr: int = 0, h_ptr: int = 0,
                    params: L.PlannerParams | None = None, asynchronous: bool = False):
        flags = L.FLAG_DEVICE_PTRS | (L.FLAG_ASYNC if asynchronous else 0)
        v = lambda q: C.c_void_p(q) if q else None  # noqa: E731
        pp = params if params is not None else L.default_planner_params(dt=self.params.dt)
        self._call("mpcq_plan_batch", self._h, C.byref(pp), int(batch), ops, int(k), v(state_ptr), v(v_cur_ptr),
                                        v(h_ptr), v(l_feet_ptr), v(v_ref_ptr), v(reduced_ptr), v(gait_ptr),
                                        v(rot_flag_ptr), v(h_rot_ptr), v(xref_ptr), v(fsteps_ptr), v(status_ptr),
                                        flags)

    # ------------------------------------------------------------------ device pointers
    def set_stream(self, stream_handle: int | None):
        self._call("mpcq_set_stream", self._h, C.c_void_p(stream_handle or 0))

    def set_slice(self, slice_iters: int):
        """Sliced batch solves (mpcq_set_slice): beyond 16 stages each batch solve suspends the
        instances still iterating after ``slice_iters`` ADMM iterations and resumes them in a
        second launch, the farthest from convergence first, to their end -- bit-identical
        outputs, a shorter dispatch tail.  0: off."""
        self._call("mpcq_set_slice", self._h, int(slice_iters))

    def solve_device(self, batch: int, xref_ptr: int, fsteps_ptr: int, f0_ptr: int, status_ptr: int,
                     iters_ptr: int = 0, x_ptr: int = 0, y_ptr: int = 0, mode: int = L.MODE_UPDATE,
                     warm_x_ptr: int = 0, warm_y_ptr: int = 0, info_ptr: int = 0,
                     asynchronous: bool = False, order_by_class: bool = False):
        flags = (L.FLAG_DEVICE_PTRS | (L.FLAG_ASYNC if asynchronous else 0)
                 | (L.FLAG_ORDER_BY_CLASS if order_by_class else 0))
        v = lambda q: C.c_void_p(q) if q else None  # noqa: E731
        self._call("mpcq_solve_batch", self._h, int(batch), v(xref_ptr), v(fsteps_ptr), mode, v(warm_x_ptr),
                                         v(warm_y_ptr), None, v(f0_ptr), v(x_ptr), v(y_ptr), None, v(status_ptr),
                                         v(iters_ptr), v(info_ptr), flags)

    def last_kernel_ms(self):
        f = C.c_double()
        s = C.c_double()
        self._call("mpcq_last_kernel_ms", self._h, C.byref(f), C.byref(s))
        return f.value, s.value
