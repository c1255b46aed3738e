"""CPU: round-3 host-side pieces -- the oracle's pre-polish ADMM status (the
checker the C3 full-batch GPU test compares info[3] against), the synthetic gait
tables at every horizon 4..64 (odd ones included), and bench.py's headline /
companion options."""
import numpy as np
import pytest


def test_oracle_reports_admm_status_before_polish(oracle, golden32):
    g, N = golden32, 32
    # max_iter far below convergence: the ADMM exits at max_iter (or inaccurate); polish = 2
    # may then upgrade the status, and admm_status keeps the ADMM's own exit code
    p2 = oracle.default_params(polish=2, polish_rounds=8, polish_refine_iter=10, max_iter=100)
    p0 = oracle.default_params(max_iter=100)
    upgraded = 0
    for b in range(4):
        r2 = oracle.qp_solve(N, g["Ax"][b], g["l"][b], g["u"][b], params=p2)
        r0 = oracle.qp_solve(N, g["Ax"][b], g["l"][b], g["u"][b], params=p0)
        assert r0["admm_status"] == r0["status"] and r0["polish"] == 0
        assert r2["admm_status"] == r0["status"]          # the same ADMM run underneath
        assert r2["iters"] == r0["iters"] == 100
        if r2["status"] == 1 and r2["admm_status"] != 1:
            upgraded += 1
            assert r2["polish"] == 1
    assert upgraded > 0
    # the batch entry point carries the same fields
    sb = oracle.solve_batch(g["xref"][:4], g["fsteps"][:4], 0, params=p2, nthreads=2)
    assert set(("admm_status", "polish", "rho_updates")) <= set(sb)
    assert (sb["admm_status"] != 1).all() and (sb["iters"] == 100).all()


@pytest.mark.parametrize("N", list(range(4, 65)))
def test_gait_tables_cover_the_horizon(N):
    import mpcq.synth as S
    for gait in S.GAITS + ("static",):
        t = S.gait_table(gait, N)
        d = t[:, 0]
        k = int(np.flatnonzero(d == 0)[0])
        assert d[:k].sum() == N and (d[:k] >= 1).all()
        for off in (1, N // 2, N - 1):
            r = S.rolled_table(gait, N, off)
            dr = r[:, 0]
            kr = int(np.flatnonzero(dr == 0)[0])
            assert dr[:kr].sum() == N


def test_bench_headline_options(monkeypatch):
    import sys
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.headline == "reference" and a.companion == 1
    monkeypatch.setattr(sys, "argv", ["bench.py", "--polish"])
    assert bench.parse().headline == "accuracy"
    monkeypatch.setattr(sys, "argv", ["bench.py", "--no-polish", "--companion", "0"])
    a = bench.parse()
    assert a.headline == "reference" and a.companion == 0
    assert bench.MODES["reference"] == {} and bench.MODES["accuracy"]["polish"] == 2
