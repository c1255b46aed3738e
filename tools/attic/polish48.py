"""Debug: polish at N = 48 (global-workspace layout) against the oracle and x*."""
import sys
import numpy as np
sys.path[:0] = ['/root/repo', '/root/repo/mpc-tsid_amd']
import mpcq  # noqa: E402
from oracle import oracle as O  # noqa: E402
for N in (32, 48):
    d = np.load('/root/repo/tests/golden/golden_horizons.npz')
    if N == 32:
        g = dict(np.load('/root/repo/tests/golden/golden_n32.npz'))
    else:
        g = {k[4:]: d[k] for k in d.files if k.startswith('n48_')}
    for rounds in (1, 8):
        over = dict(polish=2, polish_rounds=rounds, polish_refine_iter=10)
        with mpcq.Engine(N, **over) as e:
            r = e.qp_solve(g["Ax"][:5], g["l"][:5], g["u"][:5])
        p = O.default_params(**over)
        for b in range(5):
            o = O.qp_solve(N, g["Ax"][b], g["l"][b], g["u"][b], params=p)
            print(f"N={N} rounds={rounds} b={b}: gpu st {r['status'][b]} it {r['iters'][b]} pol {r['polish'][b]} "
                  f"rounds {r['polish_rounds'][b] if 'polish_rounds' in r else '-'} |f-f*| "
                  f"{np.abs(r['x'][b][12*N:] - g['x_star'][b][12*N:]).max():.2e} | oracle st {o['status']} "
                  f"|f-f*| {np.abs(o['x'][12*N:] - g['x_star'][b][12*N:]).max():.2e} "
                  f"|x_gpu-x_or| {np.abs(r['x'][b] - o['x']).max():.2e}", flush=True)
