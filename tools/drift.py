"""Where the GPU's solution leaves the oracle's, per horizon.

    python tools/drift.py [--horizons 16 48 64]

For the reference-captured QPs of each horizon (tests/golden), runs the engine and
the oracle with max_iter = 1, 2, 5, 10, 25, ... (adaptive rho at its default, so the
factorisations are the ones of the real solve) and prints the largest difference of
the solutions relative to their scale, max |x - x_oracle| / max(1, max |x|), per
max_iter: the first row is one KKT solve (the factorisation's own rounding), the rest
show how the ADMM iteration carries it.  Then a warm-started closed loop (sessions,
6 ticks) per horizon with the per-tick difference.
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mpc-tsid_amd"), REPO, os.path.join(REPO, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--horizons", type=int, nargs="+", default=[16, 48, 64])
    a = ap.parse_args()
    import mpcq
    from conftest import load_golden, GOLDEN
    from oracle import oracle as O
    O.build()
    fx = {}
    for name in ("golden_horizons.npz", "golden_horizons_r3.npz", "golden_horizons_r4.npz"):
        d = np.load(os.path.join(GOLDEN, name))
        for N in d["horizons"]:
            pre = f"n{int(N)}_"
            fx[int(N)] = {k[len(pre):]: d[k] for k in d.files if k.startswith(pre)}
    fx[16] = load_golden(16)
    fx[32] = load_golden(32)
    for N in a.horizons:
        g = fx[N]
        B = g["Ax"].shape[0]
        print(f"N = {N}: {B} reference QPs")
        for mi in (1, 2, 5, 10, 25, 50, 100, 200, 400, 800, 4000):
            with mpcq.Engine(N, max_iter=mi) as e:
                r = e.qp_solve(g["Ax"], g["l"], g["u"])
            worst, wabs, agree = 0.0, 0.0, 0
            for b in range(B):
                o = O.qp_solve(N, g["Ax"][b], g["l"][b], g["u"][b], params=O.default_params(max_iter=mi))
                d = np.abs(r["x"][b] - o["x"]).max()
                worst = max(worst, d / max(1.0, np.abs(o["x"]).max()))
                wabs = max(wabs, d)
                agree += int(o["iters"] == r["iters"][b])
            print(f"  max_iter {mi:5d}: max |x - x_oracle| {wabs:.2e} (relative to scale {worst:.2e}), "
                  f"iterations equal {agree}/{B}, iters {r['iters'].tolist()}")
        # warm-started closed loop from the host (the session test's inputs)
        from test_gpu_session import _gaits, _inputs
        Bs, T = 12, 6
        gaits = _gaits(Bs, N)
        rng = np.random.default_rng(11 + N)
        with mpcq.Engine(N, dual_warm=1) as eng, mpcq.Session(eng, Bs, gait0=gaits) as sess:
            ors = [O.Session(N, gaits[b], params=O.default_params(dual_warm=1)) for b in range(Bs)]
            for k in range(T):
                state, l_feet, v_ref = _inputs(rng, Bs, k)
                red = (np.arange(Bs) % 5 == 0).astype(np.int32)
                sess.tick(v_ref, state=state, l_feet=l_feet, reduced=red, k=k)
                for b, o in enumerate(ors):
                    o.tick(k, v_ref[b], state=state[b], l_feet=l_feet[b], reduced=bool(red[b]))
                x = sess.read(mpcq.SV_X)
                it = sess.read(mpcq.SV_ITERS)
                dx = max(float(np.abs(x[b] - o.x).max()) for b, o in enumerate(ors))
                rel = max(float(np.abs(x[b] - o.x).max() / max(1.0, np.abs(o.x).max())) for b, o in enumerate(ors))
                same = sum(int(it[b] == o.iters) for b, o in enumerate(ors))
                print(f"  session tick {k}: max |x - x_oracle| {dx:.2e} (relative {rel:.2e}), iterations equal "
                      f"{same}/{Bs}, median iters {np.median(it):.0f}")


if __name__ == "__main__":
    main()
