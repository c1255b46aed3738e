import sys
import numpy as np
sys.path[:0] = ['/root/repo', '/root/repo/mpc-tsid_amd']
import mpcq
d = np.load('/root/repo/tests/golden/golden_horizons.npz')
for N in (24, 28, 48):
    g = {k[len(f'n{N}_'):]: d[k] for k in d.files if k.startswith(f'n{N}_')}
    for ri in (10, 20, 40):
        with mpcq.Engine(N, polish=2, polish_rounds=8, polish_refine_iter=ri) as e:
            r = e.qp_solve(g["Ax"], g["l"], g["u"])
        err = [np.abs(r['x'][b][12*N:] - g['x_star'][b][12*N:]).max() for b in range(len(r['x']))]
        print(N, ri, ' '.join(f'{x:.1e}' for x in err), flush=True)
