"""GPU parity: the HIP engine (libmpcq.so through its C ABI) against the oracle
and the reference-generated golden fixtures.  Run with -m gpu on an MI355X."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FORM_TOL = 1e-13  # formulation (relative, ulp-level: FMA contraction on the GPU)
X_TOL = 1e-9      # GPU vs oracle solutions (same algorithm, same data; observed 1.5e-11)


@pytest.fixture(scope="module")
def mpcq():
    import mpcq as M
    return M


@pytest.fixture(scope="module")
def eng16(mpcq):
    e = mpcq.Engine(16)
    yield e
    e.close()


@pytest.fixture(scope="module")
def eng32(mpcq):
    e = mpcq.Engine(32)
    yield e
    e.close()


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert np.array_equal(np.isinf(a), np.isinf(b))
    fa, fb = np.where(np.isinf(a), 0, a), np.where(np.isinf(b), 0, b)
    return float((np.abs(fa - fb) / np.maximum(1.0, np.abs(fb))).max(initial=0))


@pytest.mark.parametrize("N", [16, 32])
@pytest.mark.parametrize("mode", [0, 1])
def test_formulation_vs_reference(N, mode, eng16, eng32, golden16, golden32):
    e, g = (eng16, golden16) if N == 16 else (eng32, golden32)
    sfx = "" if mode == 0 else "_setup"
    r = e.formulate(g["xref"], g["fsteps"], mode)
    assert (r["status"] == 0).all()
    err = max(_rel(r["Ax"], g["Ax" + sfx]), _rel(r["l"], g["l" + sfx]), _rel(r["u"], g["u" + sfx]))
    print(f"N={N} mode={mode} formulation max rel err vs reference {err:.2e}")
    assert err <= FORM_TOL


def test_formulation_vs_oracle_synthetic(eng16, oracle, mpcq):
    b = mpcq.synth.make_batch(256, 16, gaits=mpcq.synth.GAITS, seed=11)
    r = eng16.formulate(b["xref"], b["fsteps"], 0)
    worst = 0.0
    for i in range(0, 256, 7):
        Ax, l, u = oracle.formulate(b["xref"][i], b["fsteps"][i], 0)
        worst = max(worst, _rel(r["Ax"][i], Ax), _rel(r["l"][i], l), _rel(r["u"][i], u))
    assert worst <= FORM_TOL, worst


def test_bad_gait_status(eng16, golden16, mpcq):
    r = eng16.formulate(np.repeat(golden16["bad_xref"][None], 3, 0), golden16["bad_fsteps"], 0)
    assert (r["status"] == mpcq.STATUS_BAD_GAIT).all()
    s = eng16.solve(np.repeat(golden16["bad_xref"][None], 3, 0), golden16["bad_fsteps"], 0)
    assert (s["status"] == mpcq.STATUS_BAD_GAIT).all()
    assert np.isnan(s["f0"]).all()


@pytest.mark.parametrize("N", [16, 32])
def test_qp_solve_vs_oracle(N, eng16, eng32, golden16, golden32, oracle):
    """Same OSQP-0.6 algorithm on the same QP data: statuses and iteration
    counts identical on every instance, x within X_TOL (observed 1.5e-11)."""
    e, g = (eng16, golden16) if N == 16 else (eng32, golden32)
    r = e.qp_solve(g["Ax"], g["l"], g["u"])
    B = g["Ax"].shape[0]
    same_it = 0
    errs = []
    for b in range(B):
        o = oracle.qp_solve(N, g["Ax"][b], g["l"][b], g["u"][b])
        same_it += int(o["iters"] == r["iters"][b])
        errs.append(np.abs(r["x"][b] - o["x"]).max())
        assert r["status"][b] == o["status"], (b, r["status"][b], o["status"])
    errs = np.array(errs)
    print(f"N={N}: iteration counts equal on {same_it}/{B}; max|x-x_oracle| {errs.max():.2e} "
          f"median {np.median(errs):.2e}; iters {np.median(r['iters'])}")
    assert same_it == B
    assert errs.max() < X_TOL


def test_fused_vs_oracle(eng16, oracle, mpcq):
    b = mpcq.synth.make_batch(64, 16, gaits=mpcq.synth.GAITS, seed=5)
    r = eng16.solve(b["xref"], b["fsteps"], 0)
    o = oracle.solve_batch(b["xref"], b["fsteps"], 0, nthreads=8)
    assert np.array_equal(r["status"], o["status"])
    assert np.array_equal(r["iters"], o["iters"])
    err = np.abs(r["f0"] - o["f0"]).max(axis=1)
    print(f"fused: max|f0-f0_oracle| {err.max():.2e} median {np.median(err):.2e}")
    assert err.max() < X_TOL


def _certified(xref, fsteps, x, y):
    from oracle import certify
    fstar, kkt, ok = certify.certified_forces(xref, fsteps, x, y)
    assert ok.all(), kkt.max()
    return fstar


def test_headline_c2_full_batch(mpcq, oracle):
    """BASELINE C2 exactly as bench.py runs it (1024 instances, seed 2, trot, polish on):
    every instance solved, statuses / iteration counts / polish outcome equal to the
    oracle's on every instance, forces within 1e-6 of each QP's KKT-certified optimum
    (observed 3.3e-10) and within X_TOL of the oracle's polished forces."""
    from mpcq import shard
    b = shard.shard_batch(1024, 1, 0, 16, ("trot",), seed=2)
    over = dict(polish=2, polish_rounds=8, polish_refine_iter=10)
    with mpcq.Engine(16, **over) as e:
        r = e.solve(b["xref"], b["fsteps"], 0, want_y=True)
    assert (r["status"] == mpcq.STATUS_SOLVED).all()
    o = oracle.solve_batch(b["xref"], b["fsteps"], 0, params=oracle.default_params(**over), nthreads=16)
    assert np.array_equal(r["status"], o["status"])
    assert np.array_equal(r["iters"], o["iters"])
    assert (r["polish"] == 1).all()
    assert np.array_equal(r["polish"], o["polish"])
    assert np.array_equal(r["admm_status"], o["admm_status"])
    fstar = _certified(b["xref"], b["fsteps"], r["x"], r["y"])
    d_star = np.abs(r["f0"] - fstar).max()
    d_ora = np.abs(r["f0"] - o["f0"]).max()
    print(f"C2 full batch: max|f0 - f0*| {d_star:.2e}, max|f0 - f0_oracle| {d_ora:.2e}, "
          f"iters median {np.median(r['iters'])} max {r['iters'].max()}")
    assert d_star < 1e-8  # observed 3.3e-10
    assert d_ora < X_TOL


def test_headline_c3_full_batch(mpcq, oracle):
    """BASELINE C3 exactly as bench.py's accuracy mode runs it (1024 instances, N=32,
    seed 2, trot, polish=2): statuses, iteration counts, the ADMM's own exit status
    and the polish outcome equal to the oracle's on every instance -- including the
    instances whose ADMM stops at max_iter and that polish=2 upgrades to SOLVED
    (an engine extension: OSQP 0.6 polishes only after SOLVED) -- and forces within
    1e-8 of each QP's KKT-certified optimum (observed 3.4e-9 in round 2)."""
    from mpcq import shard
    b = shard.shard_batch(1024, 1, 0, 32, ("trot",), seed=2)
    over = dict(polish=2, polish_rounds=8, polish_refine_iter=10)
    with mpcq.Engine(32, **over) as e:
        r = e.solve(b["xref"], b["fsteps"], 0, want_y=True)
    o = oracle.solve_batch(b["xref"], b["fsteps"], 0, params=oracle.default_params(**over), nthreads=16)
    assert np.array_equal(r["status"], o["status"])
    assert np.array_equal(r["iters"], o["iters"])
    assert np.array_equal(r["admm_status"], o["admm_status"])
    assert np.array_equal(r["polish"], o["polish"])
    assert (r["status"] == mpcq.STATUS_SOLVED).all()
    upgraded = (r["admm_status"] != mpcq.STATUS_SOLVED) & (r["status"] == mpcq.STATUS_SOLVED)
    at_max = r["iters"] == 4000
    # the ADMM's exits at max_iter: SOLVED_INACCURATE (round 3: 51 of 53, the other two meet eps at
    # the last check), all of them upgraded by polish = 2
    assert upgraded.sum() > 0 and np.isin(r["admm_status"][at_max], (1, 2, -2)).all()
    assert upgraded[at_max].sum() == (r["admm_status"][at_max] != 1).sum()
    fstar = _certified(b["xref"], b["fsteps"], r["x"], r["y"])
    dfo = np.abs(r["f0"] - fstar).max(axis=1)
    d_ora = np.abs(r["f0"] - o["f0"]).max()
    print(f"C3 full batch: {int(upgraded.sum())} instances upgraded by polish ({int(at_max.sum())} at max_iter, ADMM "
          f"statuses {dict(zip(*np.unique(r['admm_status'], return_counts=True)))}); "
          f"max|f0 - f0*| {dfo.max():.2e} (upgraded ones {dfo[upgraded].max():.2e}), "
          f"max|f0 - f0_oracle| {d_ora:.2e}")
    assert dfo.max() < 1e-8
    assert d_ora < 1e-8


def test_admm_c2_full_batch_vs_oracle(eng16, mpcq, oracle):
    """C2 with polish off (the reference's own settings): statuses and iteration
    counts equal to the oracle's on all 1024 instances; the two-instances-per-CU,
    two-round schedule of the full launch changes nothing."""
    from mpcq import shard
    b = shard.shard_batch(1024, 1, 0, 16, ("trot",), seed=2)
    r = eng16.solve(b["xref"], b["fsteps"], 0)
    o = oracle.solve_batch(b["xref"], b["fsteps"], 0, nthreads=16)
    assert np.array_equal(r["status"], o["status"])
    assert np.array_equal(r["iters"], o["iters"])
    assert np.abs(r["f0"] - o["f0"]).max() < X_TOL


def test_c5_size_launch(eng16, mpcq, oracle):
    """A C5-sized launch (32768 mixed-gait instances, 64 rounds of the grid): every
    instance solved; a strided sample of 512 equals the oracle (status, iterations,
    forces within X_TOL)."""
    from mpcq import shard
    b = shard.shard_batch(32768, 1, 0, 16, ("trot", "bound", "pace"), seed=5)
    r = eng16.solve(b["xref"], b["fsteps"], 0, want_x=False)
    assert np.isin(r["status"], (1, 2)).all(), np.unique(r["status"], return_counts=True)
    sel = np.arange(0, 32768, 64)
    o = oracle.solve_batch(b["xref"][sel], b["fsteps"][sel], 0, nthreads=16)
    assert np.array_equal(r["status"][sel], o["status"])
    assert np.array_equal(r["iters"][sel], o["iters"])
    assert np.abs(r["f0"][sel] - o["f0"]).max() < X_TOL


def test_c4_full_size_launch_and_rank_shard(eng16, mpcq, oracle):
    """BASELINE C4 at its real size on one GPU (65536 trot instances, bench.py's seed 2,
    128 rounds of the grid): every instance solved; a strided sample of 512 equals the
    oracle (status, iterations, forces within X_TOL).  Then rank 3's shard of the 8-GPU
    split (8192 instances, generated alone as a rank does) launched by itself: bit for
    bit the same rows as the whole launch."""
    from mpcq import shard
    total = 65536
    b = shard.shard_batch(total, 1, 0, 16, ("trot",), seed=2)
    r = eng16.solve(b["xref"], b["fsteps"], 0, want_x=False)
    assert np.isin(r["status"], (1, 2)).all(), np.unique(r["status"], return_counts=True)
    sel = np.arange(0, total, 128)
    o = oracle.solve_batch(b["xref"][sel], b["fsteps"][sel], 0, nthreads=16)
    assert np.array_equal(r["status"][sel], o["status"])
    assert np.array_equal(r["iters"][sel], o["iters"])
    err = np.abs(r["f0"][sel] - o["f0"]).max()
    assert err < X_TOL
    lo, hi = shard.shard_bounds(total, 8, 3)
    s = shard.shard_batch(total, 8, 3, 16, ("trot",), seed=2)
    assert np.array_equal(s["xref"], b["xref"][lo:hi]) and np.array_equal(s["fsteps"], b["fsteps"][lo:hi],
                                                                             equal_nan=True)
    rs = eng16.solve(s["xref"], s["fsteps"], 0, want_x=False)
    for k in ("f0", "status", "iters"):
        assert np.array_equal(rs[k], r[k][lo:hi], equal_nan=True), k
    print(f"C4 65536: max|f0 - f0_oracle| on 512 {err:.2e}; iters median {np.median(r['iters'])} "
          f"max {r['iters'].max()}; rank-3 shard of 8 bit-identical")


def test_nonfinite_input(eng16, golden16, mpcq):
    Ax = golden16["Ax"][:2].copy()
    Ax[1, 100] = np.nan
    r = eng16.qp_solve(Ax, golden16["l"][:2], golden16["u"][:2])
    assert r["status"][0] == mpcq.STATUS_SOLVED
    assert r["status"][1] == mpcq.STATUS_NONFINITE
    assert np.isnan(r["x"][1]).all()


@pytest.mark.parametrize("N", [16, 32])
def test_polish_reaches_optimum(N, golden16, golden32, oracle, mpcq):
    """Accurate mode (polish=2, 8 active-set rounds): the GPU's forces land on the
    exact optimum x* of the reference's QP (certified by its KKT residuals in
    gen_golden.py) -- independently of the ADMM path -- as the oracle's polish
    does.  The GPU solves each active-set QP by the method of multipliers on its
    own factorisation; tolerance POLISH_TOL on the forces."""
    POLISH_TOL = 1e-8
    g = golden16 if N == 16 else golden32
    over = dict(polish=2, polish_rounds=8, polish_refine_iter=10)
    with mpcq.Engine(N, **over) as e:
        r = e.qp_solve(g["Ax"], g["l"], g["u"])
    p = oracle.default_params(**over)
    B = g["Ax"].shape[0]
    d_star, d_ora = [], []
    for b in range(B):
        o = oracle.qp_solve(N, g["Ax"][b], g["l"][b], g["u"][b], params=p)
        assert r["status"][b] == o["status"] == 1, (b, r["status"][b], o["status"])
        assert r["polish"][b] == 1, (b, r["polish"][b], o["polish"])
        d_star.append(np.abs(r["x"][b][12 * N:] - g["x_star"][b][12 * N:]).max())
        d_ora.append(np.abs(r["x"][b] - o["x"]).max())
    print(f"N={N} polish: max|f - f*| {max(d_star):.2e} (median {np.median(d_star):.2e}), "
          f"max|x - x_oracle| {max(d_ora):.2e}")
    assert max(d_star) < POLISH_TOL
    assert max(d_ora) < POLISH_TOL


def test_polish_osqp_default_mode(golden16, oracle, mpcq):
    """polish=1 (OSQP's single active-set guess after SOLVED).  The GPU solves the
    guessed equality QP to convergence (refinement against the true residuals);
    OSQP's 3 delta-regularised refinements -- restated by the oracle -- stop
    ~1e-4 short on these QPs and are sometimes rejected.  So: the GPU accepts
    wherever the oracle does, and its accepted points sit on x*."""
    g = golden16
    with mpcq.Engine(16, polish=1) as e:
        r = e.qp_solve(g["Ax"], g["l"], g["u"])
    p = oracle.default_params(polish=1)
    B = g["Ax"].shape[0]
    acc_gpu = acc_ora = 0
    worst = 0.0
    for b in range(B):
        o = oracle.qp_solve(16, g["Ax"][b], g["l"][b], g["u"][b], params=p)
        assert r["status"][b] == o["status"]
        if o["polish"] == 1:
            assert r["polish"][b] == 1, b
        acc_ora += o["polish"] == 1
        if r["polish"][b] == 1:
            acc_gpu += 1
            worst = max(worst, np.abs(r["x"][b][192:] - g["x_star"][b][192:]).max())
    print(f"polish=1: accepted on {acc_gpu}/{B} (oracle {acc_ora}/{B}), accepted max|f - f*| {worst:.2e}")
    assert acc_gpu >= acc_ora
    assert worst < 1e-8


def test_infeasibility_and_bad_bounds_vs_oracle(eng16, golden16, oracle, mpcq):
    """OSQP 0.6's primal-infeasibility detection (a swing force held at 0 and asked
    for fz >= 10 N) and l > u rejection: statuses (-3 / -13) and iteration counts
    equal to the oracle's on every instance, x NaN as osqp's store_solution, and
    the untouched feasible instances of the same launch unaffected; then
    max_iter around the detection point (MAX_ITER_REACHED vs -3 at the final
    check) in the engine's own launches."""
    from test_infeasibility import infeasible_instance
    N = 16
    Ax, L, U, kinds = [], [], [], []
    for b in range(0, 50, 3):
        inst = infeasible_instance(golden16, b)
        if inst is not None:
            Ax.append(inst[0]); L.append(inst[1]); U.append(inst[2]); kinds.append("infeasible")
        Ax.append(golden16["Ax"][b]); L.append(golden16["l"][b]); U.append(golden16["u"][b]); kinds.append("ok")
    lb = golden16["l"][1].copy()
    lb[24 * N + 3] = 1.0  # friction row with u = 0 < l
    Ax.append(golden16["Ax"][1]); L.append(lb); U.append(golden16["u"][1]); kinds.append("l>u")
    Ax, L, U = np.array(Ax), np.array(L), np.array(U)
    r = eng16.qp_solve(Ax, L, U)
    for i, kind in enumerate(kinds):
        o = oracle.qp_solve(N, Ax[i], L[i], U[i])
        assert r["status"][i] == o["status"], (i, kind, r["status"][i], o["status"])
        assert r["iters"][i] == o["iters"], (i, kind, r["iters"][i], o["iters"])
        want = {"infeasible": mpcq.STATUS_PRIMAL_INFEASIBLE, "ok": mpcq.STATUS_SOLVED,
                "l>u": mpcq.STATUS_BAD_BOUNDS}[kind]
        assert r["status"][i] == want, (i, kind)
        if kind == "ok":
            assert np.abs(r["x"][i] - o["x"]).max() < X_TOL
        else:
            assert np.isnan(r["x"][i]).all()
    inf_idx = [i for i, k in enumerate(kinds) if k == "infeasible"][:4]
    for mi in (60, 100, 101, 110):
        with mpcq.Engine(16, max_iter=mi) as e:
            rr = e.qp_solve(Ax[inf_idx], L[inf_idx], U[inf_idx])
        po = oracle.default_params(max_iter=mi)
        for j, i in enumerate(inf_idx):
            o = oracle.qp_solve(N, Ax[i], L[i], U[i], params=po)
            assert rr["status"][j] == o["status"] and rr["iters"][j] == o["iters"], (mi, i)


@pytest.mark.parametrize("dual_warm", [0, 1])
def test_dual_warm_vs_oracle(golden16, oracle, mpcq, dual_warm):
    """Two ticks per instance: a cold solve of QP a, then QP b warm-started from it
    (x, y, rho) under both dual carry-overs; iterations equal to the oracle's and
    x within W_TOL, y within Y_RTOL relative on every instance (observed 2e-9 and
    1.6e-8: the warm start carries the first solve's rounding into the second, and
    ADMM's duals converge more slowly than its primal)."""
    W_TOL, Y_RTOL = 1e-8, 1e-6
    g, N = golden16, 16
    B = 24
    a_idx, b_idx = np.arange(B), (np.arange(B) + 7) % g["Ax"].shape[0]
    with mpcq.Engine(N, dual_warm=dual_warm) as e:
        r1 = e.qp_solve(g["Ax"][a_idx], g["l"][a_idx], g["u"][a_idx])
        r2 = e.qp_solve(g["Ax"][b_idx], g["l"][b_idx], g["u"][b_idx], warm_x=r1["x"], warm_y=r1["y"],
                        rho=r1["rho"])
    p = oracle.default_params(dual_warm=dual_warm)
    for i in range(B):
        o1 = oracle.qp_solve(N, g["Ax"][a_idx[i]], g["l"][a_idx[i]], g["u"][a_idx[i]], params=p)
        o2 = oracle.qp_solve(N, g["Ax"][b_idx[i]], g["l"][b_idx[i]], g["u"][b_idx[i]], params=p,
                             warm_x=o1["x"], warm_y=o1["y"], rho=o1["rho"])
        assert r2["iters"][i] == o2["iters"], (i, r2["iters"][i], o2["iters"])
        assert np.abs(r2["x"][i] - o2["x"]).max() < W_TOL
        assert np.abs(r2["y"][i] - o2["y"]).max() < Y_RTOL * max(1.0, np.abs(o2["y"]).max())
