"""Dispatch model of a batch launch: does a two-phase (resumable) schedule beat
index-order dispatch?  

    python tools/dispatch_model.py

Iteration counts of the C2 / C3 batches (seed 2, trot) come from the oracle
(identical to the GPU's, tests/test_gpu_parity.py); per-iteration times are
tools/iterbench.py's (N = 16: 1.893 us alone, 2.307 co-resident with two
instances per CU; N = 32: 3.25 us, one per CU); per-instance overheads
(scaling, factorisations, polish) are rough constants.  The hardware is modelled
as dispatching workgroups in index order into the first free slot.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))


def iteration_counts():
    from oracle import oracle as O
    import mpcq
    out = {}
    for N in (16, 32):
        b = mpcq.synth.make_batch(1024, N, gaits=("trot",), seed=2)
        out[f"n{N}"] = O.solve_batch(b["xref"], b["fsteps"], 0, nthreads=os.cpu_count() or 1)["iters"]
    return out


def sim(work_us_alone, S, CUs=256, co=1.0):
    """work in 'alone' microseconds per instance; index-order dispatch into free slots;
    co = slowdown factor when the CU holds S>1 busy instances (event-driven, exact)."""
    n = len(work_us_alone)
    nxt, t = 0, 0.0
    rem = np.zeros((CUs, S))
    busy = np.zeros((CUs, S), bool)
    while True:
        # dispatch
        for c in range(CUs):
            for s in range(S):
                if not busy[c, s] and nxt < n:
                    rem[c, s] = work_us_alone[nxt]
                    busy[c, s] = True
                    nxt += 1
        if not busy.any():
            return t
        nb = busy.sum(axis=1, keepdims=True)
        rate = np.where(nb > 1, 1.0 / co, 1.0)
        # advance to the next completion
        tt = np.where(busy, rem / rate, np.inf).min()
        t += tt
        rem = np.where(busy, rem - tt * rate, 0.0)
        busy &= rem > 1e-9


def two_phase(it, K, per_it, S, co, ovh, resume_ovh):
    w1 = np.minimum(it, K) * per_it + ovh
    t1 = sim(w1, S, co=co)
    left = it[it > K] - K
    w2 = left * per_it + resume_ovh
    t2 = sim(w2, S, co=co) if len(left) else 0.0
    return t1, t2, len(left)


def main():
    d = iteration_counts()
    for N, per_it, S, co, ovh, rov in ((16, 1.893, 2, 2.307 / 1.893, 200.0, 60.0), (32, 3.25, 1, 1.0, 500.0, 150.0)):
        it = d[f"n{N}"].astype(float)
        base = sim(it * per_it + ovh, S, co=co)
        print(f"N={N}: single launch model {base/1e3:.2f} ms; sum-work bound {(it*per_it+ovh).sum()/256/S/1e3:.2f}")
        for K in (400, 600, 800, 1000, 1200, 1500, 2000):
            t1, t2, nl = two_phase(it, K, per_it, S, co, ovh, rov)
            print(f"  K={K}: phase1 {t1/1e3:.2f} + phase2 {t2/1e3:.2f} ({nl} resumed) = {(t1+t2)/1e3:.2f} ms")
        # longest first (oracle knowledge)
        o = np.argsort(-it)
        print(f"  LPT (iteration counts known) {sim((it*per_it+ovh)[o], S, co=co)/1e3:.2f} ms")


if __name__ == "__main__":
    main()
