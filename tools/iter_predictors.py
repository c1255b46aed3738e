"""Does any input feature predict a QP's ADMM iteration count?  (A longest-first
dispatch of a cold batch would need one: DESIGN.md section 5.)

    python tools/iter_predictors.py

Oracle iteration counts of the bench's C2 / C3 batches against the sampled
inputs (gait phase = roll offset, reference velocities); Spearman rank
correlations.  Round 6: the gait itself on C5's rank-0 shard at 8 GPUs (4096 of
32768, trot / bound / pace interleaved) -- what MPCQ_FLAG_ORDER_BY_CLASS orders by
(mpcq_order.hip).  CPU only.
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

# C5 rank-0 shard (bench.py --config c5 --batch 4096): iterations by gait, and the dispatch model
# (tools/dispatch_model.py sim: two instances per CU, the r05 per-iteration times) for index order,
# gait classes by their mean iterations (the class order) and clairvoyant longest-first
from mpcq import shard
sys.path.insert(0, '/root/repo/tools')
from dispatch_model import sim
b = shard.shard_batch(32768, 8, 0, 16, ("trot", "bound", "pace"), seed=2)
t = time.time(); o = O.solve_batch(b["xref"], b["fsteps"], 0, nthreads=8); dt = time.time() - t
it = o["iters"]; g = b["gait"]
print(f"C5 shard 4096 (rank 0 of 8): oracle {dt:.1f}s, iters median {np.median(it):.0f} max {it.max()}; "
      f"spearman(gait index, iters) {spearmanr(g, it)[0]:+.3f}")
means = {}
for q, name in enumerate(("trot", "bound", "pace")):
    s_ = it[g == q]
    means[q] = s_.mean()
    print(f"   {name:5s} n {len(s_)} mean {s_.mean():.0f} median {np.median(s_):.0f} p90 {np.percentile(s_, 90):.0f} max {s_.max()}")
w = it * 1.724 + 200.0
order = np.concatenate([np.where(g == q)[0] for q in sorted(means, key=lambda q: -means[q])])
for name, o_ in (("index order", np.arange(len(it))), ("by gait class", order), ("longest first (clairvoyant)", np.argsort(-it))):
    print(f"   dispatch model, {name:28s} {sim(w[o_], 2, co=2.06 / 1.724) / 1e3:.2f} ms")
