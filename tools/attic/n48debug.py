import sys, numpy as np
sys.path[:0] = ['/root/repo', '/root/repo/mpc-tsid_amd']
import mpcq
N = 48
d = np.load('/root/repo/tests/golden/golden_horizons.npz')
g = {k[4:]: d[k] for k in d.files if k.startswith('n48_')}
s = mpcq.synth.make_batch(96, N, gaits=mpcq.synth.GAITS, seed=100 + N)
print("gaits", [str(x) for x in s.get("gait", [])][:5] if isinstance(s, dict) else None, flush=True)
with mpcq.Engine(N) as e:
    print("1 fused golden", flush=True)
    r = e.solve(g["xref"], g["fsteps"], 0); print(r["status"], r["iters"], flush=True)
    print("2 formulate+qp synthetic", flush=True)
    f = e.formulate(s["xref"], s["fsteps"], 0); print("form status", np.unique(f["status"]), flush=True)
    r = e.qp_solve(f["Ax"], f["l"], f["u"]); print(np.unique(r["status"]), r["iters"].max(), flush=True)
    print("3 fused synthetic 8", flush=True)
    r = e.solve(s["xref"][:8], s["fsteps"][:8], 0); print(r["status"], r["iters"], flush=True)
    print("4 fused synthetic 96", flush=True)
    r = e.solve(s["xref"], s["fsteps"], 0); print(np.unique(r["status"]), r["iters"].max(), flush=True)
print("done")
