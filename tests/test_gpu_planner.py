"""GPU parity of the batched FootstepPlanner (mpcq_plan_batch, mpcq_planner.hip)
against the fixtures captured from the unmodified reference FootstepPlanner.py
and against the oracle (oracle/planner_oracle.c) on random batches.

Tolerance: gait tables, NaN patterns and the rotation state machine exact;
fsteps / xref within PLAN_TOL absolute (metres, rad, m/s).  The kernel follows
numpy's rounding order; only cos/sin (ocml vs the host libm) may differ by an
ulp, so the observed difference is 0 or a few 1e-17."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PLAN_TOL = 1e-15
GOLD = os.path.join(os.path.dirname(__file__), "golden", "planner_golden.npz")


@pytest.fixture(scope="module")
def mpcq():
    import mpcq as M
    return M


@pytest.fixture(scope="module")
def engines(mpcq):
    es = {N: mpcq.Engine(N) for N in (8, 10, 16, 24, 32, 48, 64)}
    yield es
    for e in es.values():
        e.close()


class BatchState:
    def __init__(self, gait0, N):
        B = gait0.shape[0]
        self.gait = np.ascontiguousarray(gait0, np.float64).copy()
        self.rot_flag = np.zeros(B, np.int32)
        self.h_rot = np.full(B, 0.20)
        self.xref = np.zeros((B, 12, N + 1))
        self.fsteps = np.full((B, 20, 13), np.nan)

    def plan(self, eng, ops, k, state, l_feet, v_ref, reduced=None, v_cur=None, h=None, params=None):
        return eng.plan(ops, k, state, l_feet, v_ref, self.gait, self.rot_flag, self.h_rot, self.xref,
                        self.fsteps, reduced=reduced, v_cur=v_cur, h=h, params=params)


def _close(a, b, tol=PLAN_TOL):
    a, b = np.asarray(a), np.asarray(b)
    assert np.array_equal(np.isnan(a), np.isnan(b))
    d = np.abs(np.where(np.isnan(a), 0, a) - np.where(np.isnan(b), 0, b))
    assert d.max(initial=0) <= tol, d.max()
    return float(d.max(initial=0)), float((d == 0).mean())


@pytest.mark.parametrize("N", [8, 16, 24, 32, 48, 64])
def test_planner_vs_reference_fixtures(mpcq, engines, N):
    """Every scenario of planner_golden.npz runs as one instance of a batch,
    tick by tick as processing.py:81-131 drives the reference."""
    G = np.load(GOLD)
    eng = engines[N]
    S, T = G[f"n{N}_state"].shape[:2]
    bs = BatchState(G[f"n{N}_gait0"], N)
    # the N = 8 / 24 fixtures ran FootstepPlanner(0.04, n_periods)
    pp = mpcq.default_planner_params(dt=float(G[f"n{N}_dt"][0])) if f"n{N}_dt" in G.files else None
    worst, exact = 0.0, []
    for j in range(T):
        a = (G[f"n{N}_state"][:, j], G[f"n{N}_l_feet"][:, j], G[f"n{N}_v_ref"][:, j])
        red = G[f"n{N}_reduced"][:, j].astype(np.int32)
        if j == 0:
            assert (bs.plan(eng, mpcq.PLAN_FOOTSTEPS, 0, *a, reduced=red, params=pp) == 0).all()
        assert (bs.plan(eng, mpcq.PLAN_TICK, j, *a, reduced=red, params=pp) == 0).all()
        assert np.array_equal(bs.gait, G[f"n{N}_gait"][:, j]), j
        assert np.array_equal(bs.rot_flag, G[f"n{N}_flag"][:, j]), j
        for got, want in ((bs.fsteps, G[f"n{N}_fsteps"][:, j]), (bs.xref, G[f"n{N}_xref"][:, j]),
                          (bs.h_rot, G[f"n{N}_h_rot"][:, j])):
            d, ex = _close(got, want)
            worst = max(worst, d)
            exact.append(ex)
    print(f"N={N}: {S} scenarios x {T} ticks, max |d| = {worst:.2e}, exactly equal {np.mean(exact):.4f}")


def _random_batch(rng, B, N):
    from mpcq import synth
    gait = np.zeros((B, 20, 5))
    kinds = ("trot", "bound", "pace")
    for b in range(B):
        r = rng.random()
        if r < 0.6:
            gait[b] = synth.gait_table(kinds[b % 3], N)
        elif r < 0.95:  # random phases summing to N, random masks
            nph = int(rng.integers(1, min(12, N)))
            cuts = np.sort(rng.choice(np.arange(1, N), nph - 1, replace=False)) if nph > 1 else np.array([], int)
            d = np.diff(np.concatenate([[0], cuts, [N]]))
            gait[b, :nph, 0] = d
            gait[b, :nph, 1:] = rng.integers(0, 2, (nph, 4))
        else:  # malformed: no terminator (the reference raises)
            gait[b, :, 0] = rng.integers(1, 3, 20)
            gait[b, :, 1:] = rng.integers(0, 2, (20, 4))
    state = np.concatenate([rng.normal(0, 0.02, (B, 2)), 0.2 + rng.uniform(-.01, .01, (B, 1)),
                            rng.normal(0, 0.02, (B, 2)), np.zeros((B, 1)), rng.normal(0, 0.2, (B, 6))], axis=1)
    sh = np.array([[0.19, 0.19, -0.19, -0.19], [0.15005, -0.15005, 0.15005, -0.15005]])
    l_feet = np.concatenate([sh + rng.uniform(-.03, .03, (B, 2, 4)), rng.uniform(-.005, .005, (B, 1, 4))], axis=1)
    v_ref = np.stack([rng.uniform(-.5, 1, B), rng.uniform(-.3, .3, B), rng.choice([0, .02, .1, -.2], B),
                      rng.normal(0, .1, B), rng.normal(0, .1, B),
                      np.where(rng.random(B) < .2, 0.0, rng.uniform(-.8, .8, B))], axis=1)
    reduced = (rng.random(B) < 0.3).astype(np.int32)
    return gait, state, l_feet, v_ref, reduced


@pytest.mark.parametrize("N", [10, 16, 32, 64])
def test_planner_vs_oracle_random(mpcq, engines, N):
    from oracle import oracle as O
    rng = np.random.default_rng(77 + N)
    B = 512
    gait, state, l_feet, v_ref, reduced = _random_batch(rng, B, N)
    bs = BatchState(gait, N)
    ors = [O.Planner(N, gait[b]) for b in range(B)]
    eng = engines[N]
    bad_seen = 0
    for j, ops in enumerate((mpcq.PLAN_FOOTSTEPS, mpcq.PLAN_TICK, mpcq.PLAN_ROLL, mpcq.PLAN_REFSTATES,
                             mpcq.PLAN_TICK, mpcq.PLAN_ROLL | mpcq.PLAN_FOOTSTEPS, mpcq.PLAN_TICK)):
        v_cur = state[:, 6:] + rng.normal(0, 0.01, (B, 6)) if j == 3 else None
        st = bs.plan(eng, ops, j, state, l_feet, v_ref, reduced=reduced, v_cur=v_cur)
        for b in range(B):
            so = ors[b].plan(ops, j, state[b], l_feet[b], v_ref[b], reduced=bool(reduced[b]),
                             v_cur=None if v_cur is None else v_cur[b])
            assert st[b] == so, (j, b)
            bad_seen += so != 0
        assert np.array_equal(bs.gait, np.stack([o.gait for o in ors])), j
        assert np.array_equal(bs.rot_flag, np.concatenate([o.flag for o in ors])), j
        _close(bs.fsteps, np.stack([o.fsteps for o in ors]))
        _close(bs.xref, np.stack([o.xref for o in ors]))
        _close(bs.h_rot, np.concatenate([o.h_rot for o in ors]))
        state = state + rng.normal(0, 0.01, state.shape)
    assert bad_seen > 0  # malformed tables were exercised


@pytest.mark.parametrize("N,B", [(16, 7), (31, 5), (31, 64), (8, 1)])
def test_planner_half_wave_edges(mpcq, N, B):
    """Up to N = 31 two instances share a wave64 (32 lanes each): odd batches leave the
    last wave's second half empty, N = 31 fills every lane of a half with a column.
    Every op sequence of the random test, against the oracle."""
    from oracle import oracle as O
    rng = np.random.default_rng(900 + 10 * N + B)
    gait, state, l_feet, v_ref, reduced = _random_batch(rng, B, N)
    bs = BatchState(gait, N)
    ors = [O.Planner(N, gait[b]) for b in range(B)]
    with mpcq.Engine(N) as eng:
        for j, ops in enumerate((mpcq.PLAN_TICK, mpcq.PLAN_ROLL | mpcq.PLAN_FOOTSTEPS, mpcq.PLAN_REFSTATES,
                                 mpcq.PLAN_TICK)):
            st = bs.plan(eng, ops, j, state, l_feet, v_ref, reduced=reduced)
            for b in range(B):
                so = ors[b].plan(ops, j, state[b], l_feet[b], v_ref[b], reduced=bool(reduced[b]))
                assert st[b] == so, (j, b)
            assert np.array_equal(bs.gait, np.stack([o.gait for o in ors])), j
            assert np.array_equal(bs.rot_flag, np.concatenate([o.flag for o in ors])), j
            _close(bs.fsteps, np.stack([o.fsteps for o in ors]))
            _close(bs.xref, np.stack([o.xref for o in ors]))
            state = state + rng.normal(0, 0.01, state.shape)


def test_planner_api_errors(mpcq, engines):
    eng = engines[16]
    bs = BatchState(np.zeros((2, 20, 5)), 16)
    st = np.zeros((2, 12))
    with pytest.raises(mpcq.MpcqError):
        bs.plan(eng, 0, 0, st, np.zeros((2, 3, 4)), np.zeros((2, 6)))
    with pytest.raises(mpcq.MpcqError):
        bs.plan(eng, 8, 0, st, np.zeros((2, 3, 4)), np.zeros((2, 6)))
    with pytest.raises(ValueError):
        eng.plan(mpcq.PLAN_TICK, 0, st, np.zeros((2, 3, 4)), np.zeros((2, 6)), bs.gait[:1], bs.rot_flag,
                 bs.h_rot, bs.xref, bs.fsteps)
