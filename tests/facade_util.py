"""Test-only: an engine stand-in that runs the oracle (CPU), with the Engine
method signatures the façade uses.  Lets the façade's host logic (warm start,
dual / rho carry-over, fsteps mutation, first-call forces) be checked without a
GPU, and gives the GPU façade test its expected values."""
import numpy as np


class OracleEngine:
    def __init__(self, O, n_steps=16, **overrides):
        import mpcq
        self.O = O
        self.n_steps = n_steps
        self.params = mpcq.default_params(**overrides)
        self.oparams = O.default_params(**overrides)
        self.calls = []

    def formulate(self, xref, fsteps, mode=0):
        xref, fsteps = np.asarray(xref), np.asarray(fsteps)
        if xref.ndim == 3:  # a batch of one, as Engine.formulate takes it
            xref, fsteps = xref[0], fsteps[0]
        try:
            Ax, l, u = self.O.formulate(xref, fsteps, mode, self.oparams)
            st = 0
        except ValueError:
            n, m, nnz = self.O.dims(self.n_steps)
            Ax, l, u, st = np.zeros(nnz), np.zeros(m), np.zeros(m), -11
        return dict(Ax=Ax[None], l=l[None], u=u[None], status=np.array([st], np.int32))

    def solve(self, xref, fsteps, mode=0, warm_x=None, warm_y=None, rho=None, want_x=True, want_y=True):
        """The fused tick (formulate + qp_solve) on the oracle, Engine.solve's signature."""
        f = self.formulate(xref[0], fsteps[0], mode)
        if f["status"][0] != 0:
            n, m = 24 * self.n_steps, 44 * self.n_steps
            return dict(f0=np.full((1, 12), np.nan), x=np.full((1, n), np.nan), y=np.full((1, m), np.nan),
                        rho=np.array([np.nan]), status=f["status"], iters=np.zeros(1, np.int32))
        r = self.qp_solve(f["Ax"], f["l"], f["u"], warm_x, warm_y, rho)
        r["f0"] = r["x"][:, 12 * self.n_steps:12 * self.n_steps + 12]
        return r

    def qp_solve(self, Ax, l, u, warm_x=None, warm_y=None, rho=None):
        self.calls.append(dict(warm_x=None if warm_x is None else np.array(warm_x),
                               warm_y=None if warm_y is None else np.array(warm_y), rho=rho))
        r = self.O.qp_solve(self.n_steps, Ax[0], l[0], u[0], self.oparams, warm_x, warm_y, rho)
        return dict(x=r["x"][None], y=r["y"][None], status=np.array([r["status"]]),
                    iters=np.array([r["iters"]]), rho=np.array([r["rho"]]))


class Planner:
    """The two attributes MPC_Wrapper.solve reads from a FootstepPlanner (MPC_Wrapper.py:103)."""

    def __init__(self, xref, fsteps):
        self.xref = np.array(xref)
        self.fsteps = np.array(fsteps)
