"""Generate tests/golden/planner_golden.npz (run in the build container only).

    python tests/golden/gen_planner_golden.py

Imports the UNMODIFIED reference /root/reference/FootstepPlanner.py and drives
it tick by tick exactly as the reference control loop does
(processing.py:81-89 then :131):

    tick 0:  update_fsteps(0, ...)            compute_footsteps only (k == 0)
             update_fsteps(1, ...)            roll + compute_footsteps
             getRefStates(0, ...)
    tick j:  update_fsteps(j*k_mpc + 1, ...)  roll + compute_footsteps
             getRefStates(j, ...)

with v_cur = [lV; lW] and h = lC[2] (processing.py:81-82).  Two in-process
shims are needed and change no reference file: ``np.int = int`` (removed in
numpy 2) and an empty ``pybullet`` module (imported at FootstepPlanner.py:4,
not used by these methods).

Scenarios (seeded): trot from the constructor (create_walking_trot), bound /
pace / random 20-row gait tables written into ``planner.gait``, one and two
gait periods (N = 16 / 32), random local-frame states and feet, joystick
commands that walk the height/rotation state machine (v_ref[2] beyond and
inside the 0.05 dead band), v_ref[5] = 0 on some ticks (the dx / dy branch of
FootstepPlanner.py:336-343), ``reduced`` on some ticks.  Per tick the inputs
and the planner's state after the tick are stored (gait, fsteps, xref,
flag_rotation_command, h_rotation_command).  Malformed tables: whether the
reference raises.

Only data leaves this script: inputs and expected outputs.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
T_TICKS = 24
K_MPC = 20


def import_reference_planner():
    np.int = int  # FootstepPlanner.py:56,193,... use the alias numpy 2 removed
    sys.modules.setdefault("pybullet", types.ModuleType("pybullet"))
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import FootstepPlanner  # noqa: E402  (the unmodified reference file)
    return FootstepPlanner


MASKS = {
    "bound": ((1, 1, 1, 1), (1, 1, 0, 0), (1, 1, 1, 1), (0, 0, 1, 1)),
    "pace": ((1, 1, 1, 1), (1, 0, 1, 0), (1, 1, 1, 1), (0, 1, 0, 1)),
}


def table(kind: str, n_periods: int, rng, dt: float = 0.02) -> np.ndarray:
    g = np.zeros((20, 5))
    half = int(0.5 * 0.32 / dt)  # as create_walking_trot (FootstepPlanner.py:193-214)
    N = 2 * half * n_periods
    if kind in MASKS:
        for i in range(n_periods):
            g[4 * i:4 * i + 4, 0] = (1, half - 1, 1, half - 1)
            g[4 * i:4 * i + 4, 1:] = MASKS[kind]
    elif kind == "random":
        # random phases (durations sum to N), random contact masks, repeated masks allowed
        nph = int(rng.integers(2, 9))
        cuts = np.sort(rng.choice(np.arange(1, N), nph - 1, replace=False))
        d = np.diff(np.concatenate([[0], cuts, [N]]))
        g[:nph, 0] = d
        g[:nph, 1:] = rng.integers(0, 2, (nph, 4))
    elif kind == "static":
        g[0, 0] = N
        g[0, 1:] = 1
    else:
        raise ValueError(kind)
    return g


def draw_inputs(rng, tick):
    lC = np.array([[0.0], [0.0], [0.2027682 + rng.uniform(-0.01, 0.01)]])
    abg = np.array([[rng.normal(0, 0.02)], [rng.normal(0, 0.02)], [0.0]])
    lV = rng.normal(0, 0.2, (3, 1))
    lW = rng.normal(0, 0.2, (3, 1))
    sh = np.array([[0.19, 0.19, -0.19, -0.19], [0.15005, -0.15005, 0.15005, -0.15005]])
    l_feet = np.vstack([sh + rng.uniform(-0.03, 0.03, (2, 4)), rng.uniform(-0.005, 0.005, (1, 4))])
    v_ref = np.zeros((6, 1))
    v_ref[0, 0] = rng.uniform(-0.5, 1.0)
    v_ref[1, 0] = rng.uniform(-0.3, 0.3)
    # height command: walk the state machine (beyond, inside and exactly at the dead band)
    v_ref[2, 0] = rng.choice([0.0, 0.0, 0.02, -0.03, 0.08, -0.1, 0.05])
    v_ref[3, 0] = rng.normal(0, 0.1)
    v_ref[4, 0] = rng.normal(0, 0.1)
    v_ref[5, 0] = 0.0 if rng.random() < 0.25 else rng.uniform(-0.5, 0.5)
    reduced = bool(rng.random() < 0.3)
    return lC, abg, lV, lW, l_feet, v_ref, reduced


def run_scenario(FP, kind: str, n_periods: int, seed: int, dt: float = 0.02):
    rng = np.random.default_rng(seed)
    pl = FP.FootstepPlanner(dt, n_periods)
    if kind != "trot":
        pl.gait = table(kind, n_periods, rng, dt)
    N = pl.n_steps
    rec = {k: [] for k in ("state", "l_feet", "v_ref", "reduced", "gait", "fsteps", "xref", "flag", "h_rot")}
    gait0 = pl.gait.copy()
    for j in range(T_TICKS):
        lC, abg, lV, lW, l_feet, v_ref, reduced = draw_inputs(rng, j)
        v_cur = np.vstack((lV, lW))
        if j == 0:
            pl.update_fsteps(0, l_feet, v_cur, v_ref, lC[2, 0], None, None, reduced)
        pl.update_fsteps(j * K_MPC + 1, l_feet, v_cur, v_ref, lC[2, 0], None, None, reduced)
        pl.getRefStates(float(j), pl.T_gait, lC, abg, lV, lW, v_ref, h_ref=0.2027682)
        rec["state"].append(np.concatenate([lC, abg, lV, lW]).ravel())
        rec["l_feet"].append(l_feet.copy())
        rec["v_ref"].append(v_ref.ravel().copy())
        rec["reduced"].append(reduced)
        rec["gait"].append(pl.gait.copy())
        rec["fsteps"].append(pl.fsteps.copy())
        rec["xref"].append(pl.xref.copy())
        rec["flag"].append(pl.flag_rotation_command)
        rec["h_rot"].append(pl.h_rotation_command)
    out = {k: np.array(v) for k, v in rec.items()}
    out["gait0"] = gait0
    return N, out


def raises(fn):
    try:
        fn()
    except Exception as e:  # noqa: BLE001
        return type(e).__name__
    return ""


def main():
    FP = import_reference_planner()
    groups = {}
    kinds = ("trot", "bound", "pace", "random", "random", "random", "static")
    sid = 0
    for n_periods in (1, 2):
        for kind in kinds:
            N, out = run_scenario(FP, kind, n_periods, seed=5000 + sid)
            sid += 1
            groups.setdefault(N, []).append((kind, out))
    # other horizons: dt = 0.04 (N = 8 per period: n_periods 1 and 3 -> N = 8, 24),
    # three and (round 3) four periods at dt = 0.02 (N = 48, 64); keys n<N>_*, the
    # N = 16 / 32 ones unchanged
    for dt, n_periods in ((0.04, 1), (0.04, 3), (0.02, 3), (0.02, 4)):
        for kind in ("trot", "bound", "random", "static"):
            N, out = run_scenario(FP, kind, n_periods, seed=7000 + sid, dt=dt)
            sid += 1
            out["dt"] = np.float64(dt)
            groups.setdefault(N, []).append((kind, out))
    arrs = {}
    for N, lst in groups.items():
        arrs[f"n{N}_kind"] = np.array([k for k, _ in lst])
        for key in lst[0][1]:
            arrs[f"n{N}_{key}"] = np.stack([o[key] for _, o in lst])
    # malformed tables (FootstepPlanner.py:405 roll: next(...)[0] on the 0.0 default;
    # compute_footsteps: self.gait[20, 0] past the table)
    pl = FP.FootstepPlanner(0.02, 1)
    bad = np.zeros((20, 5))
    bad[:, 0] = 1.0
    bad[::2, 1:] = 1.0
    lf = np.vstack([pl.shoulders, np.zeros((1, 4))])
    v = np.zeros((6, 1))

    def do_roll():
        pl.gait = bad.copy()
        pl.roll()

    def do_foot():
        pl.gait = bad.copy()
        pl.compute_footsteps(lf, v, v, 0.2, False)

    arrs["bad_gait"] = bad
    arrs["bad_roll_raises"] = np.array(raises(do_roll))
    arrs["bad_footsteps_raises"] = np.array(raises(do_foot))
    path = os.path.join(HERE, "planner_golden.npz")
    np.savez_compressed(path, **arrs)
    print("wrote", path, os.path.getsize(path), "bytes;", arrs["bad_roll_raises"], arrs["bad_footsteps_raises"])
    for N, lst in groups.items():
        fl = np.stack([o["flag"] for _, o in lst])
        print(f"N={N}: scenarios {[k for k, _ in lst]}, rotation flags seen {sorted(set(fl.ravel().tolist()))}")


if __name__ == "__main__":
    main()
