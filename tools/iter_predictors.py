"""Does any input feature predict a QP's ADMM iteration count?  (A longest-first
dispatch of a cold batch would need one: DESIGN.md section 5.)

    python tools/iter_predictors.py

Oracle iteration counts of the bench's C2 / C3 batches against the sampled
inputs (gait phase = roll offset, reference velocities); Spearman rank
correlations.  CPU only.
"""
import sys, numpy as np, time
sys.path[:0] = ['/root/repo', '/root/repo/mpc-tsid_amd']
import mpcq
from oracle import oracle as O
O.build()
from scipy.stats import spearmanr
for seed, N in ((2, 16), (5, 16), (2, 32)):
    b = mpcq.synth.make_batch(1024, N, gaits=("trot",), seed=seed)
    t = time.time(); o = O.solve_batch(b["xref"], b["fsteps"], 0, nthreads=8); dt = time.time() - t
    it = o["iters"]
    v = b["v_ref"]
    feats = {"offset": b["offset"], "|vx|": np.abs(v[:, 0]), "vx": v[:, 0], "|vy|": np.abs(v[:, 1]), "|wz|": np.abs(v[:, 5]),
             "|v|": np.linalg.norm(v[:, [0, 1, 5]], axis=1), "offset%4": b["offset"] % 4, "offset%8": b["offset"] % 8}
    print(f"seed {seed} N {N}: oracle {dt:.1f}s, iters median {np.median(it):.0f} max {it.max()} p90 {np.percentile(it,90):.0f}")
    for k, f in feats.items():
        print(f"   {k:10s} spearman {spearmanr(f, it)[0]:+.3f}")
    # mean iterations per offset
    print("   iters by offset:", [int(np.mean(it[b['offset'] == q])) for q in range(N)])
    np.savez(f"/tmp/pred_{seed}_{N}.npz", iters=it, offset=b["offset"], v_ref=v)
