"""Repeat the same launch many times and compare the results bit for bit
(statuses, iterations, forces) — a race or an uninitialised read shows up as a
difference between launches.

    python tools/determinism.py [--reps 10]"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import mpcq
    for N, B, gaits, seed, over in ((16, 1024, ("trot",), 2, dict(polish=2, polish_rounds=8, polish_refine_iter=10)),
                                   (16, 1024, ("trot",), 2, {}), (8, 1024, mpcq.synth.GAITS, 8, {}),
                                   (32, 512, ("trot",), 3, {})):
        src = mpcq.synth.make_batch(B, N, gaits=gaits, seed=seed)
        with mpcq.Engine(N, **over) as e:
            ref = None
            bad = 0
            for r in range(a.reps):
                out = e.solve(src["xref"], src["fsteps"], 0)
                cur = (out["status"].copy(), out["iters"].copy(), out["f0"].copy())
                nan = int(np.isnan(cur[2]).sum())
                if ref is None:
                    ref = cur
                    same = True
                else:
                    same = all(np.array_equal(x, y, equal_nan=True) for x, y in zip(ref, cur))
                bad += (not same) or nan > 0
                print(f"N={N} B={B} {'polish' if over else 'admm'} rep {r}: same {same} nan {nan} "
                      f"iters median {np.median(cur[1])} min {cur[1].min()}", flush=True)
            print(f"N={N}: {bad} bad of {a.reps}", flush=True)


if __name__ == "__main__":
    main()
