"""Debug: N = 8 statuses / NaNs after few iterations (MPCQ_LIB_VARIANT selects a build)."""
import sys
import numpy as np
sys.path[:0] = ['/root/repo', '/root/repo/mpc-tsid_amd']
import mpcq  # noqa: E402
d = np.load('/root/repo/tests/golden/golden_horizons.npz')
for N in (4, 8, 12):
    g = {k[len(f'n{N}_'):]: d[k] for k in d.files if k.startswith(f'n{N}_')}
    for mi in (1, 2, 25, 26, 4000):
        with mpcq.Engine(N, max_iter=mi) as e:
            r = e.qp_solve(g["Ax"], g["l"], g["u"])
        print(N, mi, r["status"].tolist(), r["iters"].tolist(), int(np.isnan(r["x"]).sum()), flush=True)
