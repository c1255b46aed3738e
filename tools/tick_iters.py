"""Closed-loop sessions: are a robot's ADMM iteration counts stable from one tick
to the next, and would dispatching the solve longest-previous-first shorten the
launch?  

    python tools/tick_iters.py [--robots 1024] [--ticks 30]

Runs bench.py's tick workload (virtual robots, seeded v_ref), reads every
robot's iteration count after each tick, and feeds tools/dispatch_model.py's
index-order dispatch model with (a) the robot order, (b) the order sorted by the
previous tick's counts, (c) the order sorted by the tick's own counts (LPT, the
bound), next to the measured solve-kernel time.
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", type=int, default=1024)
    ap.add_argument("--ticks", type=int, default=30)
    ap.add_argument("--N", type=int, default=16)
    ap.add_argument("--seed", type=int, default=2)
    a = ap.parse_args()
    import torch
    import mpcq
    from mpcq import synth
    from dispatch_model import sim
    dev = torch.device("cuda", 0)
    B, N = a.robots, a.N
    rng = np.random.default_rng(a.seed)
    gaits = np.stack([synth.gait_table("trot", N) for _ in range(B)])
    v_ref = np.stack([rng.uniform(-.5, 1, B), rng.uniform(-.3, .3, B), np.zeros(B), np.zeros(B),
                      np.zeros(B), rng.uniform(-.5, .5, B)], axis=1)
    vr = torch.from_numpy(v_ref).to(dev)
    per_it, co, ovh = (1.893, 2.307 / 1.893, 100.0) if N <= 16 else (3.25, 1.0, 250.0)
    S = 2 if N <= 16 else 1
    with mpcq.Engine(N) as eng:
        sess = mpcq.Session(eng, B, gait0=gaits)
        prev = None
        rows = []
        for k in range(a.ticks):
            sess.tick_device(vr.data_ptr(), k=k, asynchronous=False)
            torch.cuda.synchronize()
            it = sess.read(mpcq.SV_ITERS).astype(float)
            solve_ms = eng.last_kernel_ms()[1]
            w = it * per_it + ovh
            m_idx = sim(w, S, co=co) / 1e3
            m_lpt = sim(w[np.argsort(-it, kind="stable")], S, co=co) / 1e3
            if prev is not None:
                m_prev = sim(w[np.argsort(-prev, kind="stable")], S, co=co) / 1e3
                r = float(np.corrcoef(prev, it)[0, 1]) if it.std() > 0 and prev.std() > 0 else float("nan")
            else:
                m_prev, r = float("nan"), float("nan")
            rows.append((k, solve_ms, np.median(it), it.max(), r, m_idx, m_prev, m_lpt))
            prev = it
            print(f"tick {k:2d}: solve {solve_ms:6.3f} ms | iters median {np.median(it):6.0f} max {it.max():5.0f} | "
                  f"corr(prev) {r:5.2f} | model: index {m_idx:6.3f}  by-prev {m_prev:6.3f}  LPT {m_lpt:6.3f} ms",
                  flush=True)
        sess.close()
    rs = np.array(rows[2:], float)
    print(f"ticks 2..{a.ticks - 1}: measured {rs[:, 1].mean():.3f} ms; model index {rs[:, 5].mean():.3f}, "
          f"by-prev {rs[:, 6].mean():.3f}, LPT {rs[:, 7].mean():.3f} ms; mean corr {np.nanmean(rs[:, 4]):.2f}")


if __name__ == "__main__":
    main()
