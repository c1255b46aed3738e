"""Generate the committed golden fixtures (run in the build container only).

    python tests/golden/gen_golden.py            # writes tests/golden/golden_n16.npz, golden_n32.npz
    python tests/golden/gen_golden.py horizons   # writes tests/golden/golden_horizons.npz
                                                 # (N = 4, 8, 12, 20, 24, 28 and 48; keys n<N>_<field>)
    python tests/golden/gen_golden.py horizons_r3  # golden_horizons_r3.npz: N = 5, 6, 10, 13, 33,
                                                   # 36, 40, 57, 64
    python tests/golden/gen_golden.py horizons_r4  # golden_horizons_r4.npz: N = 49, 50

What it does, per instance:
1. Inputs: seeded synthetic (xref, fsteps) from mpcq.synth (trot / bound /
   pace, plus the static C1 case and the test_motionless.py case).
2. Formulation: imports the UNMODIFIED reference /root/reference/MPC.py and
   runs MPC.run(0, ...) then MPC.run(1, ...) exactly as MPC_Wrapper does
   (MPC_Wrapper.py:103), capturing what MPC.call_solver hands to OSQP
   (MPC.py:414 setup -> P, setup-mode A/l/u; MPC.py:419 update -> update-mode
   A.data/l/u).  Three in-process shims are needed and change no reference
   file: ``np.int = int`` (removed in numpy 2), a ``utils`` module carrying
   only a getSkew (utils.py:179-185; the real utils imports pybullet /
   pinocchio, absent here), and an ``osqp`` recorder (the osqp wheel is
   absent; it records arguments and returns x = 0).
3. Optimum: the QP is strictly convex (P diagonal > 0), so x* is unique.  It
   is computed here, independently of oracle/ and of the GPU code, by an
   OSQP-style ADMM warm phase followed by primal-dual active-set polishing on
   the UNSCALED KKT with sparse LU and iterative refinement, and certified by
   its KKT residuals (primal feasibility, stationarity, multiplier signs,
   complementarity), stored next to x*.  (scipy's HiGHS QP was tried and
   rejected: it stops ~4e-3 away from x* in force space because the force
   weight 1e-5 makes the objective nearly flat there.)

Only data leaves this script: inputs and expected outputs.  No reference
source is copied into the fixtures.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as sla

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))
from mpcq import synth  # noqa: E402

INF = 1e30


# --------------------------------------------------------------------------- reference import
class _OsqpRecorder:
    def __init__(self):
        self.calls = []
        self.n = None

    def setup(self, **kw):
        self.calls.append(("setup", {k: (v.copy() if hasattr(v, "copy") else v) for k, v in kw.items()}))
        self.n = kw["P"].shape[0]

    def update_settings(self, **kw):
        self.calls.append(("settings", dict(kw)))

    def update(self, **kw):
        self.calls.append(("update", {k: np.array(v, copy=True) for k, v in kw.items()}))

    def warm_start(self, **kw):
        self.calls.append(("warm_start", {k: np.array(v, copy=True) for k, v in kw.items()}))

    def solve(self):
        return types.SimpleNamespace(x=np.zeros(self.n))


def import_reference_mpc():
    np.int = int  # numpy>=1.24 removed the alias MPC.py uses (MPC.py:337,351,628-630)
    osqp = types.ModuleType("osqp")
    osqp.OSQP = _OsqpRecorder
    sys.modules["osqp"] = osqp
    ut = types.ModuleType("utils")

    def getSkew(a):
        return np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]], dtype=a.dtype)

    ut.getSkew = getSkew
    sys.modules["utils"] = ut
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import MPC  # noqa: E402  (the unmodified reference file)
    return MPC


def reference_qps(MPC, xref, fsteps, dt=0.02):
    """run(0) then run(1) as MPC_Wrapper.run_MPC_synchronous does; return the
    setup-mode and update-mode QP data handed to osqp."""
    N = xref.shape[1] - 1
    mpc = MPC.MPC(dt, N, 0.32)
    mpc.run(0, xref.copy(), fsteps.copy())
    mpc.run(1, xref.copy(), fsteps.copy())
    calls = mpc.prob.calls
    setup = [c for c in calls if c[0] == "setup"][0][1]
    upd = [c for c in calls if c[0] == "update"][0][1]
    settings = [c[1] for c in calls if c[0] == "settings"]
    A = setup["A"]
    return dict(P=setup["P"].diagonal().copy(), indptr=A.indptr.copy(), indices=A.indices.copy(),
                Ax_setup=A.data.copy(), l_setup=setup["l"].copy(), u_setup=setup["u"].copy(),
                Ax=upd["Ax"], l=upd["l"], u=upd["u"], settings=settings)


def reference_raises(MPC, xref, fsteps):
    try:
        reference_qps(MPC, xref, fsteps)
    except Exception as e:  # noqa: BLE001
        return type(e).__name__
    return ""


# --------------------------------------------------------------------------- exact optimum
def _admm(Pd, A, l, u, iters=6000, rho=0.1, sigma=1e-6, alpha=1.6):
    """Scaled OSQP-style ADMM, used only to find the active set."""
    n, m = A.shape[1], A.shape[0]
    As = A.tocsc().astype(float)
    D = np.ones(n)
    E = np.ones(m)
    Ps = Pd.copy()
    for _ in range(15):
        dn = np.maximum(np.abs(Ps), abs(As).max(axis=0).toarray().ravel())
        en = abs(As).max(axis=1).toarray().ravel()
        dn[dn < 1e-4] = 1.0
        en[en < 1e-4] = 1.0
        dt_, et_ = 1 / np.sqrt(dn), 1 / np.sqrt(en)
        Ps = dt_ * Ps * dt_
        As = sp.diags(et_) @ As @ sp.diags(dt_)
        D *= dt_
        E *= et_
    ls, us = E * np.maximum(l, -INF), E * np.minimum(u, INF)
    R = np.where(us - ls < 1e-4, 1e3 * rho, rho)
    K = sla.splu((sp.diags(Ps + sigma) + As.T @ sp.diags(R) @ As).tocsc())
    x, z, y = np.zeros(n), np.zeros(m), np.zeros(m)
    for k in range(1, iters + 1):
        xt = K.solve(sigma * x + As.T @ (R * z - y))
        zt = As @ xt
        x = alpha * xt + (1 - alpha) * x
        zr = alpha * zt + (1 - alpha) * z
        zn = np.clip(zr + y / R, ls, us)
        y = y + R * (zr - zn)
        z = zn
        if k % 200 == 0:
            pr = np.abs((As @ x - z) / E).max()
            dr = np.abs((Ps * x + As.T @ y) / D).max()
            if pr < 1e-10 and dr < 1e-10:
                break
            ax, zz, aty = As @ x, z, As.T @ y
            rn = rho * np.sqrt((np.abs(ax - zz).max() / max(np.abs(ax).max(), np.abs(zz).max(), 1e-30)) /
                               (np.abs(Ps * x + aty).max() / max(np.abs(Ps * x).max(), np.abs(aty).max(), 1e-30) + 1e-30))
            rn = min(max(rn, 1e-6), 1e6)
            if rn > 5 * rho or rn < rho / 5:
                rho = rn
                R = np.where(us - ls < 1e-4, 1e3 * rho, rho)
                K = sla.splu((sp.diags(Ps + sigma) + As.T @ sp.diags(R) @ As).tocsc())
    return D * x, E * z, E * y


def kkt_residuals(Pd, A, l, u, x, y):
    """(primal infeasibility, stationarity, multiplier-sign violation, complementarity)."""
    z = A @ x
    prim = max(np.maximum(l - z, 0).max(), np.maximum(z - u, 0).max())
    stat = np.abs(Pd * x + A.T @ y).max()
    lo_gap = np.where(np.isfinite(l), z - l, np.inf)
    hi_gap = np.where(np.isfinite(u), u - z, np.inf)
    # y < 0 only at a lower bound, y > 0 only at an upper bound
    sign = max(np.maximum(y, 0)[hi_gap > 1e-9].max(initial=0.0), np.maximum(-y, 0)[lo_gap > 1e-9].max(initial=0.0))
    comp = max((np.maximum(-y, 0) * np.minimum(lo_gap, 1e3)).max(), (np.maximum(y, 0) * np.minimum(hi_gap, 1e3)).max())
    return np.array([prim, stat, sign, comp])


def _eq_solve(Pd, A, l, u, lo, hi, delta, refine):
    n, m = A.shape[1], A.shape[0]
    act = lo | hi
    Aa = A[act]
    b = np.where(lo, l, u)[act]
    ma = Aa.shape[0]
    K = sp.bmat([[sp.diags(Pd + delta), Aa.T], [Aa, -delta * sp.eye(ma)]]).tocsc()
    K0 = sp.bmat([[sp.diags(Pd), Aa.T], [Aa, None]]).tocsc()
    F = sla.splu(K)
    rhs = np.concatenate([np.zeros(n), b])
    sol = F.solve(rhs)
    for _ in range(refine):
        sol = sol + F.solve(rhs - K0 @ sol)
    xp = sol[:n]
    yp = np.zeros(m)
    yp[act] = sol[n:]
    return xp, yp


def exact_optimum(Pd, A, l, u, rounds=40, delta=1e-9, refine=30):
    """Active-set refinement of an ADMM guess: each round solves the equality
    QP on the current set, then drops rows whose multiplier has the wrong sign
    and adds rows the solution violates; the best KKT-residual round is kept."""
    A = A.tocsc()
    x, z, y = _admm(Pd, A, l, u)
    rownz = np.diff(A.tocsr().indptr) > 0
    eq = (u - l) < 1e-12
    lo = (z - l < -y) & rownz
    hi = (~lo) & (u - z < y) & rownz
    best = None
    seen = set()
    for _ in range(rounds):
        key = (lo.tobytes(), hi.tobytes())
        if key in seen:
            break
        seen.add(key)
        xp, yp = _eq_solve(Pd, A, l, u, lo, hi, delta, refine)
        res = kkt_residuals(Pd, A, l, u, xp, yp)
        if best is None or res.max() < best[2].max():
            best = (xp, yp, res)
        if res.max() < 1e-13:
            break
        zp = A @ xp
        tol = 1e-12
        keep_lo = lo & ((yp <= tol) | eq)
        keep_hi = hi & ((yp >= -tol) | eq)
        add_lo = (zp < l - tol) & rownz & ~keep_hi
        add_hi = (zp > u + tol) & rownz & ~keep_lo
        lo, hi = keep_lo | add_lo, keep_hi | add_hi
    return best


# --------------------------------------------------------------------------- driver
def build(N: int, per_gait: int, seed: int, extra=True):
    MPC = import_reference_mpc()
    insts = []
    for gi, g in enumerate(synth.GAITS):
        b = synth.make_batch(per_gait, N, gaits=(g,), seed=seed + 7 * gi)
        for i in range(per_gait):
            insts.append((b["xref"][i], b["fsteps"][i], gi))
    if extra:
        c1 = synth.make_batch(1, N, gaits=("trot",), static=True)
        insts.append((c1["xref"][0], c1["fsteps"][0], 3))
        mo = synth.motionless(N)
        insts.append((mo["xref"][0], mo["fsteps"][0], 4))
    out = {k: [] for k in ("xref", "fsteps", "gait", "Ax", "l", "u", "Ax_setup", "l_setup", "u_setup",
                           "x_star", "y_star", "kkt")}
    P = indptr = indices = None
    for (xr, fs, g) in insts:
        q = reference_qps(MPC, xr, fs)
        P, indptr, indices = q["P"], q["indptr"], q["indices"]
        A = sp.csc_matrix((q["Ax"], indices, indptr), shape=(44 * N, 24 * N))
        x, y, res = exact_optimum(P, A, q["l"], q["u"])
        for k, v in (("xref", xr), ("fsteps", fs), ("gait", g), ("Ax", q["Ax"]), ("l", q["l"]), ("u", q["u"]),
                     ("Ax_setup", q["Ax_setup"]), ("l_setup", q["l_setup"]), ("u_setup", q["u_setup"]),
                     ("x_star", x), ("y_star", y), ("kkt", res)):
            out[k].append(v)
        print(f"N={N} gait={g} kkt={res}", flush=True)
    arrs = {k: np.array(v) for k, v in out.items()}
    arrs.update(P=P, indptr=indptr, indices=indices)
    # malformed gaits: record whether the reference raises
    bad = []
    xr, fs, _ = insts[0]
    f1 = fs.copy(); f1[:, 0] = 1.0                       # no terminator row
    f2 = fs.copy(); f2[0, 0] += 3.0                      # durations sum > N
    f3 = fs.copy(); f3[0, 0] = np.nan                    # NaN duration
    for f in (f1, f2, f3):
        bad.append(f)
    arrs["bad_fsteps"] = np.array(bad)
    arrs["bad_raises"] = np.array([reference_raises(MPC, xr, f) for f in bad])
    arrs["bad_xref"] = xr
    return arrs


HORIZONS = ((4, 2, 404), (8, 4, 808), (12, 2, 1212), (20, 2, 2020), (24, 4, 2424), (28, 2, 2828), (48, 1, 4848))
# round 3: horizons that are not a multiple of 4 (phantom stage rows), odd ones (the
# two sweep chains equally long) and the global-workspace range up to n_periods = 4
# (N = 64; beyond 49 stages the constraint values leave LDS too)
HORIZONS_R3 = ((5, 1, 505), (6, 2, 606), (10, 2, 1010), (13, 1, 1313), (33, 1, 3333), (36, 1, 3636), (40, 1, 4040),
               (57, 1, 5757), (64, 1, 6464))
# round 4: the layout switch points beyond 48 stages -- N = 49 (13 waves: the F row and
# the z update's constants leave registers, the constraint values still in LDS) and
# N = 50 (the constraint values in the workspace, kAbG)
HORIZONS_R4 = ((49, 1, 4949), (50, 1, 5050))


def main_horizons():
    """The other horizons the engine compiles (N = 4j <= 32) plus N = 48 (three
    16-step periods at dt = 0.02: n_periods = 3 in FootstepPlanner.py:55)."""
    out = {}
    for N, per_gait, seed in HORIZONS:
        arrs = build(N, per_gait, seed)
        for k, v in arrs.items():
            out[f"n{N}_{k}"] = v
    path = os.path.join(HERE, "golden_horizons.npz")
    np.savez_compressed(path, horizons=np.array([h[0] for h in HORIZONS]), **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def main_horizons_r3():
    """golden_horizons_r3.npz: HORIZONS_R3, same fields and key scheme as main_horizons."""
    out = {}
    for N, per_gait, seed in HORIZONS_R3:
        arrs = build(N, per_gait, seed)
        for k, v in arrs.items():
            out[f"n{N}_{k}"] = v
    path = os.path.join(HERE, "golden_horizons_r3.npz")
    np.savez_compressed(path, horizons=np.array([h[0] for h in HORIZONS_R3]), **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def main_horizons_r4():
    """golden_horizons_r4.npz: HORIZONS_R4, same fields and key scheme as main_horizons."""
    out = {}
    for N, per_gait, seed in HORIZONS_R4:
        arrs = build(N, per_gait, seed)
        for k, v in arrs.items():
            out[f"n{N}_{k}"] = v
    path = os.path.join(HERE, "golden_horizons_r4.npz")
    np.savez_compressed(path, horizons=np.array([h[0] for h in HORIZONS_R4]), **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "horizons_r4":
        main_horizons_r4()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "horizons":
        main_horizons()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "horizons_r3":
        main_horizons_r3()
        return
    for N, per_gait, seed in ((16, 16, 1234), (32, 4, 4321)):
        arrs = build(N, per_gait, seed)
        path = os.path.join(HERE, f"golden_n{N}.npz")
        np.savez_compressed(path, **arrs)
        print("wrote", path, os.path.getsize(path), "bytes; reference raises:", arrs["bad_raises"])


if __name__ == "__main__":
    main()
