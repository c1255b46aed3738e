"""Debug: the engine after a few ADMM iterations (max_iter) against the oracle, per horizon:
which entries of x differ (indexing errors show up after one iteration).

    python tools/onestep.py [max_iter ...]     (MPCQ_LIB_VARIANT selects a build)"""
import sys

import numpy as np

sys.path[:0] = ['/root/repo', '/root/repo/mpc-tsid_amd']
import mpcq  # noqa: E402
from oracle import oracle as O  # noqa: E402

its = [int(a) for a in sys.argv[1:]] or [1, 2, 26, 101]
for N in (4, 8, 16, 32):
    if N in (16, 32):
        g = dict(np.load(f'/root/repo/tests/golden/golden_n{N}.npz'))
    else:
        d = np.load('/root/repo/tests/golden/golden_horizons.npz')
        g = {k[len(f'n{N}_'):]: d[k] for k in d.files if k.startswith(f'n{N}_')}
    for mi in its:
        with mpcq.Engine(N, max_iter=mi) as e:
            r1 = e.qp_solve(g['Ax'][:2], g['l'][:2], g['u'][:2])
        o1 = O.qp_solve(N, g['Ax'][0], g['l'][0], g['u'][0], params=O.default_params(max_iter=mi))
        d = np.abs(r1['x'][0] - o1['x'])
        bad = np.where(d > 1e-9)[0]
        print(f"N={N} max_iter={mi}: max|dx| {d.max():.3e} (states {d[:12 * N].max():.3e}, forces {d[12 * N:].max():.3e})"
              f" bad {len(bad)}: {bad[:16].tolist()}", flush=True)
