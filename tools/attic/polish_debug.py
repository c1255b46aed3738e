"""Polish diagnostics: per-instance status / polish result / rounds vs the oracle."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))
sys.path.insert(0, REPO)


def main():
    import ctypes as C
    import mpcq
    from mpcq import _lib as L
    from oracle import oracle as O
    g = dict(np.load(os.path.join(REPO, "tests", "golden", "golden_n16.npz")))
    over = dict(polish=2, polish_rounds=8, polish_refine_iter=10)
    if len(sys.argv) > 1:
        over["delta"] = float(sys.argv[1])
    B = 6
    with mpcq.Engine(16, **over) as e:
        Ax, l, u = (np.ascontiguousarray(g[k][:B]) for k in ("Ax", "l", "u"))
        x = np.empty((B, 384)); y = np.empty((B, 704)); st = np.empty(B, np.int32); it = np.empty(B, np.int32)
        ro = np.empty(B); info = np.empty((B, 4), np.int32)
        p = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
        L.check(L.lib().mpcq_qp_solve_batch(e._h, B, p(Ax), p(l), p(u), None, None, None, p(x), p(y), p(st), p(it),
                                            p(ro), p(info), 0))
    op = O.default_params(**over)
    for b in range(B):
        o = O.qp_solve(16, g["Ax"][b], g["l"][b], g["u"][b], params=op)
        print(over.get("delta", 1e-6), b, "gpu", st[b], it[b], info[b].tolist(), "| oracle", o["status"], o["iters"], o["polish"],
              "| |f-f*| gpu %.2e oracle %.2e" % (np.abs(x[b][192:] - g["x_star"][b][192:]).max(),
                                                  np.abs(o["x"][192:] - g["x_star"][b][192:]).max()))


if __name__ == "__main__":
    main()
