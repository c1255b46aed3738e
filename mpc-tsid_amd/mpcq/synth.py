"""Synthetic (xref, fsteps) batches shaped like the reference's MPC inputs.

The reference produces the MPC inputs with FootstepPlanner (OUT of the hot
path).  This module restates the parts of it that shape
those inputs so the batch bench and the parity tests run on realistic data:

* gait tables: create_walking_trot / create_bounding / create_side_walking
  (FootstepPlanner.py:207-282), one [1, N/2-1, 1, N/2-1] period per 16 steps,
  laid out in the 20-row table of FootstepPlanner.py:62-63;
* roll() (FootstepPlanner.py:401-425) applied ``offset`` times;
* getRefStates (FootstepPlanner.py:76-161) for k > 0 with the joystick's
  height/rotation state machine in its starting state (flag 0);
* compute_footsteps / compute_next_footstep (FootstepPlanner.py:284-399) with
  ``reduced=False`` and the reference's call pattern compute_next_footstep(
  v_ref, v_ref, h) (FootstepPlanner.py:325).

Sampling: v_ref = (vx~U[-.5,1], vy~U[-.3,.3], 0, 0, 0,
wz~U[-.5,.5]); x0 = (0, 0, h_ref+U[-.01,.01], N(0,.02), N(0,.02), 0,
v_ref[:3]+N(0,.05), N(0,.05)); feet at the shoulders + U[-.03,.03] in xy.
Everything is vectorised over the batch; it runs on the host (numpy).
"""
from __future__ import annotations

import numpy as np

DT = 0.02
T_GAIT = 0.32
H_REF = 0.2027682
SHOULDERS = np.array([[0.19, 0.19, -0.19, -0.19], [0.15005, -0.15005, 0.15005, -0.15005]])
K_FEEDBACK = 0.03
G = 9.81
L_MAX = 0.12
T_STANCE = 0.16

# stance masks of the 4 phases of one period, feet ordered FL, FR, HL, HR
GAIT_MASKS = {
    "trot": ((1, 1, 1, 1), (1, 0, 0, 1), (1, 1, 1, 1), (0, 1, 1, 0)),   # FootstepPlanner.py:226-229
    "bound": ((1, 1, 1, 1), (1, 1, 0, 0), (1, 1, 1, 1), (0, 0, 1, 1)),  # :251-254
    "pace": ((1, 1, 1, 1), (1, 0, 1, 0), (1, 1, 1, 1), (0, 1, 0, 1)),   # :277-280
}
GAITS = ("trot", "bound", "pace")


def period_steps(n_steps: int) -> int:
    """MPC steps per gait period for horizon n_steps: 16 (T_gait / dt at dt = 0.02)
    when N is a whole number of such periods, else one period spanning the horizon
    (the reference's N = n_periods T_gait / dt, FootstepPlanner.py:55, with
    dt = T_gait / N, e.g. N = 8 at dt = 0.04; N = 24 = 3 periods of 8 is another
    valid table, this one is the single-period choice)."""
    p = int(round(T_GAIT / DT))
    return p if n_steps % p == 0 else n_steps


def gait_table(gait: str, n_steps: int) -> np.ndarray:
    """20x5 table: [duration, stance FL, FR, HL, HR] (FootstepPlanner.py:207-231)."""
    g = np.zeros((20, 5))
    if gait == "static":
        g[0, 0] = n_steps
        g[0, 1:] = 1.0
        return g
    if n_steps < 4:
        raise ValueError(f"horizon {n_steps}: a gait period is two half periods of >= 2 steps")
    per = period_steps(n_steps)
    n_periods = n_steps // per
    if n_periods > 4:
        raise ValueError(f"horizon {n_steps}: {n_periods} periods do not fit the 20-row table")
    # an odd single-period horizon has half periods of floor(N/2) and ceil(N/2) steps
    h1, h2 = per // 2, per - per // 2
    masks = GAIT_MASKS[gait]
    for i in range(n_periods):
        g[4 * i:4 * i + 4, 0] = (1, h1 - 1, 1, h2 - 1)
        for r in range(4):
            g[4 * i + r, 1:] = masks[r]
    return g


def roll(g: np.ndarray) -> np.ndarray:
    """One step of FootstepPlanner.roll (FootstepPlanner.py:401-425)."""
    g = g.copy()
    index = int(np.flatnonzero(g[:, 0] == 0.0)[0])
    if np.array_equal(g[0, 1:], g[index - 1, 1:]):
        g[index - 1, 0] += 1.0
    else:
        g[index, 1:] = g[0, 1:]
        g[index, 0] = 1.0
    if g[0, 0] > 1.0:
        g[0, 0] -= 1.0
    else:
        g = np.roll(g, -1, axis=0)
        g[-1, :] = 0.0
    return g


def rolled_table(gait: str, n_steps: int, offset: int) -> np.ndarray:
    g = gait_table(gait, n_steps)
    for _ in range(offset):
        g = roll(g)
    return g


def ref_states(lC, abg, lV, lW, v_ref, n_steps: int, h_ref: float = H_REF) -> np.ndarray:
    """getRefStates for k > 0, flag_rotation_command == 0 (FootstepPlanner.py:94-161).

    All inputs are batched: lC, abg, lV, lW (B,3); v_ref (B,6).  Returns (B,12,N+1).
    """
    B = lC.shape[0]
    xref = np.zeros((B, 12, n_steps + 1))
    yaw = np.linspace(0, T_GAIT - DT, n_steps)[None, :] * v_ref[:, 5:6]
    vx, vy, wz = v_ref[:, 0:1], v_ref[:, 1:2], v_ref[:, 5:6]
    xref[:, 6, 1:] = vx * np.cos(yaw) - vy * np.sin(yaw)
    xref[:, 7, 1:] = vx * np.sin(yaw) + vy * np.cos(yaw)
    xref[:, 0, 1:] = DT * np.cumsum(xref[:, 6, 1:], axis=1)
    xref[:, 1, 1:] = DT * np.cumsum(xref[:, 7, 1:], axis=1)
    xref[:, 0, 1:] += lC[:, 0:1]
    xref[:, 1, 1:] += lC[:, 1:2]
    dt_vector = np.linspace(DT, T_GAIT, n_steps)
    xref[:, 5, 1:] = wz * dt_vector[None, :]
    xref[:, 11, 1:] = wz
    xref[:, 0:3, 0] = lC
    xref[:, 3:6, 0] = abg
    xref[:, 6:9, 0] = lV
    xref[:, 9:12, 0] = lW
    # joystick state machine, starting state (flag 0): z = h_ref, vz = 0
    xref[:, 2, 1:] = h_ref
    xref[:, 8, 1:] = 0.0
    return xref


def next_footstep(v_ref: np.ndarray, h: float = H_REF) -> np.ndarray:
    """compute_next_footstep(v_ref, v_ref, h) (FootstepPlanner.py:363-399). (B,3,4)."""
    B = v_ref.shape[0]
    nf = np.zeros((B, 3, 4))
    v = v_ref[:, 0:2, None]
    nf[:, 0:2, :] += T_STANCE * 0.5 * v
    nf[:, 0:2, :] += K_FEEDBACK * (v - v)
    cross = np.cross(v_ref[:, 0:3], v_ref[:, 3:6])
    nf[:, 0:2, :] += 0.5 * np.sqrt(h / G) * cross[:, 0:2, None]
    nf[:, 0:2, :] = np.clip(nf[:, 0:2, :], -L_MAX, L_MAX)
    nf[:, 0:2, :] += SHOULDERS[None]
    return nf


def footsteps(gait_tab: np.ndarray, l_feet, v_cur, v_ref, h: float = H_REF) -> np.ndarray:
    """compute_footsteps (FootstepPlanner.py:284-361) for instances sharing one table.

    gait_tab (20,5); l_feet (B,3,4); v_cur, v_ref (B,6).  Returns fsteps (B,20,13).
    """
    B = l_feet.shape[0]
    fs = np.full((B, 20, 13), np.nan)
    fs[:, :, 0] = gait_tab[None, :, 0]
    rpt = np.repeat(gait_tab[:, 1:] == 1, 3, axis=1)  # (20,12)
    lf = l_feet.transpose(0, 2, 1).reshape(B, 12)     # ravel(order='F')
    fs[:, 0, 1:][:, rpt[0]] = lf[:, rpt[0]]
    nf = None
    i = 1
    dt_cum = 0.0
    while gait_tab[i, 0] != 0:
        dt_cum += gait_tab[i - 1, 0] * DT
        keep = rpt[i - 1] & rpt[i]
        fs[:, i, 1:][:, keep] = fs[:, i - 1, 1:][:, keep]
        fs[:, i, 1:][:, ~rpt[i]] = np.nan
        land = (~rpt[i - 1]) & rpt[i]
        if land.any():
            if nf is None:
                nf = next_footstep(v_ref, h)
            w = v_ref[:, 5]
            ang = w * dt_cum
            c, s = np.cos(ang), np.sin(ang)
            R = np.zeros((B, 3, 3))
            R[:, 0, 0], R[:, 0, 1], R[:, 1, 0], R[:, 1, 1], R[:, 2, 2] = c, -s, s, c, 1.0
            safe = np.where(w != 0, w, 1.0)
            dx = np.where(w != 0, (v_cur[:, 0] * np.sin(ang) + v_cur[:, 1] * (np.cos(ang) - 1)) / safe,
                          v_cur[:, 0] * dt_cum)
            dy = np.where(w != 0, (v_cur[:, 1] * np.sin(ang) - v_cur[:, 0] * (np.cos(ang) - 1)) / safe,
                          v_cur[:, 1] * dt_cum)
            nft = R @ nf
            nft[:, 0, :] += dx[:, None]
            nft[:, 1, :] += dy[:, None]
            nft = nft.transpose(0, 2, 1).reshape(B, 12)
            fs[:, i, 1:][:, land] = nft[:, land]
        i += 1
    return fs


CHUNK = 1024  # instances per independently seeded block of a synthetic batch


def _chunk_rng(seed: int, c: int):
    """Generator of block c: block 0 is default_rng(seed) itself, so a batch of at
    most CHUNK instances is the one the earlier rounds generated."""
    return np.random.default_rng(seed if c == 0 else [seed, c])


def _make_block(rng, g0: int, B: int, N: int, gaits, static: bool, interleave: bool):
    """Instances g0 .. g0 + B - 1 of a batch, drawn from ``rng``."""
    v_ref = np.zeros((B, 6))
    if not static:
        v_ref[:, 0] = rng.uniform(-0.5, 1.0, B)
        v_ref[:, 1] = rng.uniform(-0.3, 0.3, B)
        v_ref[:, 5] = rng.uniform(-0.5, 0.5, B)
    lC = np.zeros((B, 3))
    lC[:, 2] = H_REF + (0.0 if static else rng.uniform(-0.01, 0.01, B))
    abg = np.zeros((B, 3))
    lV = v_ref[:, 0:3].copy()
    lW = np.zeros((B, 3))
    if not static:
        abg[:, 0:2] = rng.normal(0.0, 0.02, (B, 2))
        lV += rng.normal(0.0, 0.05, (B, 3))
        lW = rng.normal(0.0, 0.05, (B, 3))
    l_feet = np.zeros((B, 3, 4))
    l_feet[:, 0:2, :] = SHOULDERS[None]
    if not static:
        l_feet[:, 0:2, :] += rng.uniform(-0.03, 0.03, (B, 2, 4))
    if interleave:
        gsel = (g0 + np.arange(B)) % len(gaits)
    else:
        gsel = rng.integers(0, len(gaits), B)
    offset = np.zeros(B, np.int64) if static else rng.integers(0, N, B)
    xref = ref_states(lC, abg, lV, lW, v_ref, N)
    fsteps = np.empty((B, 20, 13))
    v_cur = np.concatenate([lV, lW], axis=1)
    for gi, gname in enumerate(gaits):
        for off in np.unique(offset[gsel == gi]):
            sel = np.flatnonzero((gsel == gi) & (offset == off))
            tab = rolled_table(gname, N, int(off))
            fsteps[sel] = footsteps(tab, l_feet[sel], v_cur[sel], v_ref[sel])
    return dict(xref=xref, fsteps=fsteps, gait=gsel, offset=offset, v_ref=v_ref)


def make_batch(batch: int, n_steps: int = 16, gaits=("trot",), seed: int = 0,
               static: bool = False, interleave: bool = True, lo: int = 0, hi: int | None = None):
    """Seeded synthetic batch, or the slice [lo, hi) of it.

    Returns dict(xref (B,12,N+1), fsteps (B,20,13), gait (B,) int index into
    ``gaits``, offset (B,) roll offset, v_ref (B,6)).  ``static=True`` gives the
    C1 case: v_ref = 0, standing state, every instance on the unrolled table.
    Mixed gaits are interleaved (instance b gets gaits[b % len(gaits)]).

    The batch is generated in blocks of CHUNK instances, block c from its own
    generator (``_chunk_rng(seed, c)``), so a slice costs only the blocks it
    touches and equals the same rows of the whole batch: a rank of a sharded run
    builds its own shard only (mpcq/shard.py).
    """
    B, N = int(batch), int(n_steps)
    hi = B if hi is None else int(hi)
    lo = int(lo)
    if not 0 <= lo <= hi <= B:
        raise ValueError(f"slice [{lo}, {hi}) of a batch of {B}")
    parts = []
    for c in range(lo // CHUNK, -(-hi // CHUNK)):
        c0, c1 = c * CHUNK, min((c + 1) * CHUNK, B)
        blk = _make_block(_chunk_rng(seed, c), c0, c1 - c0, N, gaits, static, interleave)
        a, b = max(lo, c0) - c0, min(hi, c1) - c0
        parts.append({k: v[a:b] for k, v in blk.items()})
    if not parts:
        blk = _make_block(_chunk_rng(seed, 0), 0, 0, N, gaits, static, interleave)
        return blk
    if len(parts) == 1:
        return parts[0]
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


def motionless(n_steps: int = 16) -> dict:
    """The canonical standing case of test_motionless.py:22-47 (all four feet in
    stance for the whole horizon, lV = (0, 0, 0.1), xref[8, 1:] = 0)."""
    x0 = np.array([0.0, 0.0, 0.2, 0.0, 0.0, 0.0, 0.0, 0.0, 0.1, 0.0, 0.0, 0.0])
    xref = np.repeat(x0[:, None], n_steps + 1, axis=1)
    xref[8, 1:] = 0.0
    fsteps = np.full((20, 13), np.nan)
    fsteps[:, 0] = 0.0
    fsteps[0, 0] = n_steps
    feet = np.array([[0.19, 0.19, -0.19, -0.19], [0.15005, -0.15005, 0.15005, -0.15005], [0.0] * 4])
    fsteps[0, 1:] = feet.ravel(order="F")
    return dict(xref=xref[None], fsteps=fsteps[None])
