"""Factorisation cycle count per instance (MPCQ_LIB_VARIANT=ft build, -DMPCQ_FACTIME)."""
import os, sys, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpc-tsid_amd"))
import mpcq
N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
eng = mpcq.Engine(N)
src = mpcq.synth.make_batch(1024, N, gaits=("trot",), seed=2)
info = np.empty((1024, 4), np.int32)
import ctypes as C
from mpcq import _lib as L
B=1024
f0 = np.empty((B, 12)); st = np.empty(B, np.int32); it = np.empty(B, np.int32)
xr = np.ascontiguousarray(src["xref"]); fs = np.ascontiguousarray(src["fsteps"])
p = lambda a: a.ctypes.data_as(C.c_void_p)
L.check(L.lib().mpcq_solve_batch(eng._h, B, p(xr), p(fs), 1, None, None, None, p(f0), None, None, None, p(st), p(it), p(info), 0))
fc = info[:, 2].astype(np.float64) * 256
nf = info[:, 0] + 1
per = fc / nf
print("factorisations per instance: mean %.2f max %d" % (nf.mean(), nf.max()))
print("cycles per factorisation: median %.0f min %.0f max %.0f" % (np.median(per), per.min(), per.max()))
print("slowest instance: iters %d, factorisations %d, factor cycles %.0f" % (it.max(), nf[np.argmax(it)], fc[np.argmax(it)]))
