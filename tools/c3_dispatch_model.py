"""Dispatch models of C3's launch (N = 32, one instance per CU): index order (the
hardware), a clairvoyant longest-first order, and multi-launch slicing (every launch runs
each unfinished instance for up to Q more iterations, resuming from a checkpointed iterate
after R iteration-equivalents of recomputing formulation, scaling and factorisation).

    python tools/c3_dispatch_model.py

Oracle iteration counts of the C3 batch (bench.py: 1024 instances, N = 32, trot, seed 2); 2.898 us per iteration
(r05ai), 256 CUs, a setup of 30 iteration-equivalents, greedy list scheduling.  CPU only.
"""
import os
import sys
import heapq

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mpc-tsid_amd")]
import mpcq
from oracle import oracle as O
O.build()
b = mpcq.synth.make_batch(1024, 32, gaits=("trot",), seed=2)  # bench.py --config c3 (seed 2)
it = O.solve_batch(b["xref"], b["fsteps"], 0, nthreads=min(8, os.cpu_count() or 1))["iters"].astype(float)
print('iters: median', np.median(it), 'mean', it.mean(), 'max', it.max(), 'n max', (it == it.max()).sum())
PER, CUS, SETUP = 2.898, 256, 30.0
def listsched(jobs):  # greedy list scheduling on CUS identical machines, jobs in order (durations in its)
    h = [0.0] * CUS
    heapq.heapify(h)
    for d in jobs:
        t = heapq.heappop(h); heapq.heappush(h, t + d)
    return max(h)
base = listsched(it + SETUP) * PER
print(f'index order: {base/1e3:.2f} ms; total/256 = {(it+SETUP).sum()/CUS*PER/1e3:.2f} ms; longest {((it.max()+SETUP)*PER)/1e3:.2f} ms')
lpt = listsched(np.sort(it + SETUP)[::-1]) * PER
print(f'LPT (clairvoyant): {lpt/1e3:.2f} ms ({lpt/base:.2f}x)')
for Q in (200, 400, 800, 1600):
    for R in (10.0, 30.0):
        # multi-launch: each launch runs every remaining instance for up to Q iterations
        rem = it.copy(); total = 0.0; first = True; nl = 0
        while (rem > 0).any():
            act = rem > 0
            sl = np.minimum(rem[act], Q) + (SETUP if first else R)
            total += listsched(sl) * PER + 15.0  # + a launch / compaction gap (us)
            rem[act] -= np.minimum(rem[act], Q); first = False; nl += 1
        print(f'multi-launch Q={Q} R={R:.0f}: {total/1e3:.2f} ms ({total/base:.2f}x), {nl} launches')
