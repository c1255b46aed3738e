"""Dispatch models of C2's launch beyond index order.

    python tools/slice_model.py

Iteration counts of the C2 batch from the oracle (equal to the GPU's); per-iteration
time 1.823 us alone on a CU / 2.19 us with a co-resident instance (tools/iterbench.py,
r05f); 256 CUs x 2 slots; a per-instance setup of 16 iteration-equivalents.  Policies:
index order (the hardware), a clairvoyant longest-first order, and time slicing (an
instance is suspended after Q iterations and requeued at the tail, resuming from its
checkpointed iterate after R iteration-equivalents of recomputation).  1-us steps.
"""
import collections
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mpc-tsid_amd")]

ALONE, CO, SETUP, CUS = 1.823, 2.19, 16.0, 256


def run(iters, order, Q=None, R=0.0):
    q = collections.deque((int(i), float(iters[i]) + SETUP) for i in order)
    slot = [[None, None] for _ in range(CUS)]

    def pull():
        if not q:
            return None
        i, rem = q.popleft()
        return [i, rem, Q if Q is not None else float("inf")]
    for s in range(2):
        for c in range(CUS):
            slot[c][s] = pull()
    t = 0.0
    while any(e is not None for row in slot for e in row):
        t += 1.0
        for c in range(CUS):
            rate = 1.0 / (CO if slot[c][0] is not None and slot[c][1] is not None else ALONE)
            for s in range(2):
                e = slot[c][s]
                if e is None:
                    continue
                e[1] -= rate
                e[2] -= rate
                if e[1] <= 0:
                    slot[c][s] = pull()
                elif e[2] <= 0:
                    if q:  # suspend and requeue; run to completion once nothing waits
                        q.append((e[0], e[1] + R))
                        slot[c][s] = pull()
                    else:
                        e[2] = float("inf")
    return t


def main():
    import mpcq
    from oracle import oracle as O
    O.build()
    b = mpcq.synth.make_batch(1024, 16, gaits=("trot",), seed=2)
    it = O.solve_batch(b["xref"], b["fsteps"], 0, nthreads=os.cpu_count() or 1)["iters"]
    idx = np.arange(len(it))
    base = run(it, idx)
    print(f"index order: {base / 1e3:.2f} ms")
    lpt = run(it, np.argsort(-it, kind="stable"))
    print(f"longest first (clairvoyant): {lpt / 1e3:.2f} ms ({lpt / base:.2f}x)")
    for Q in (100, 200, 400, 800):
        for R in (41.0, 5.0):
            v = run(it, idx, Q, R)
            print(f"time slicing Q = {Q} iterations, resume {R:.0f}: {v / 1e3:.2f} ms ({v / base:.2f}x)")


if __name__ == "__main__":
    main()
