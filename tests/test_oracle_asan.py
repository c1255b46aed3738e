"""CPU: the oracle's C restatements (formulation, OSQP ADMM + polish +
infeasibility detection, planner, session epilogue) under AddressSanitizer and
UndefinedBehaviorSanitizer (oracle/Makefile `asan`, -fsanitize=address,undefined
-fno-sanitize-recover=undefined; SURVEY.md §5 "host ASan/UBSan build of the
C++ CPU path").  The checks run in a child interpreter with libasan preloaded;
any report aborts it with a non-zero exit code."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = [REPO, REPO + '/mpc-tsid_amd']
from oracle import oracle as O
from mpcq import synth
for N in (4, 16, 32):
    b = synth.make_batch(6, N, gaits=synth.GAITS, seed=N)
    r = O.solve_batch(b['xref'], b['fsteps'], 0, nthreads=1)
    assert np.isin(r['status'], (1, 2)).all(), r['status']
    Ax, l, u = O.formulate(b['xref'][0], b['fsteps'][0], 1)
    p = O.default_params(polish=2, polish_rounds=8, polish_refine_iter=10)
    assert O.qp_solve(N, Ax, l, u, params=p)['status'] == 1
    # infeasible (a swing force forced to zero and to >= 10 N) and l > u
    u2 = u.copy(); u2[24 * N + 4] = -10.0; l2 = l.copy(); l2[24 * N + 4] = -np.inf
    fs = b['fsteps'][0]
    q = [f for f in range(4) if np.isnan(fs[0, 1 + 3 * f])]
    if q:
        Ax, l, u = O.formulate(b['xref'][0], fs, 0)
        u3 = u.copy(); u3[24 * N + 5 * q[0] + 4] = -10.0
        assert O.qp_solve(N, Ax, l, u3)['status'] == -3
    l4 = l.copy(); l4[3] = u[3] + 1.0
    assert O.qp_solve(N, Ax, l4, u)['status'] == -13
    # planner + session epilogue, a few ticks
    s = O.Session(N, synth.gait_table('trot', N))
    for k in range(3):
        s.tick(k, np.array([0.3, 0.0, 0.0, 0.0, 0.0, 0.1]))
print('asan-ok')
"""


@pytest.mark.timeout(600)
def test_oracle_under_asan_ubsan():
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(asan) or not os.path.exists(asan):
        pytest.skip("libasan not available")
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"], check=True)
    env = dict(os.environ, LD_PRELOAD=asan, MPCQ_ORACLE_ASAN="1",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-c", SCRIPT.replace("REPO", repr(REPO))], env=env,
                       capture_output=True, text=True, timeout=580)
    assert r.returncode == 0 and "asan-ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
