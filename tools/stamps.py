"""Per-phase cycle breakdown of the engine kernel (diagnostic build).

    MPCQ_LIB_VARIANT=stamps python tools/stamps.py [--batch 1024] [--N 16]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))
os.environ.setdefault("MPCQ_LIB_VARIANT", "stamps")

NAMES = ["prologue", "scaling", "factor", "iter:w,b,u,beta,bt", "chk:publish", "chk:primal", "iter:inward sweeps+S^-1 y",
         "iter:outward sweeps", "chk:dual", "iter:forces", "iter:z/y/x update", "chk:reduce+adapt", "epilogue", "fac:phaseP", "fac:phaseS"]
# bucket 15 (round 4): the right-hand-side phase's own work up to its barrier; bucket 3 is
# then the wait at that barrier (the slowest wave's lag).  MPCQ_STAMP_WAVE=w builds
# (tools/build_variant.sh, MPCQ_LIB_VARIANT=exp:<name>) stamp wave w instead of wave 0.
NAMES = NAMES + ["iter:w,b,u,beta,bt (own)"]
NAMES[3] = "iter:rhs barrier wait"
# the cyclic-reduction build (kCR horizons): bucket 3 is ph_rhs + its barrier, 15 the
# reduction of b + its barrier, 12 the outward sweep + the barrier after it, 7 the
# back-substitution of the odd stages + ph_recover's barrier
# the explicit-inverse build (kKI, N = 16): bucket 6 is the product, 7 the wait at its barrier
NAMES_KI = list(NAMES)
NAMES_KI[6] = "iter:Z r product (own share)"
NAMES_KI[7] = "iter:product barrier wait"
NAMES_KI[2] = "factor + Z formation"
# the nested-dissection build (kND, N = 32): 15 ph_rhs + the barrier before the sweeps, 3 the
# first rows, 6 the inward half sweep, 7 the outward half sweep (+ ph_recover's barrier wait),
# 4 the separator's terms, 5 the barrier after them, 8 the correction (4 / 5 / 8 also take the
# checks' publish / primal / dual phases, one iteration in 25)
NAMES_ND = list(NAMES)
NAMES_ND[15] = "nd:rhs + barrier"
NAMES_ND[3] = "nd:first rows"
NAMES_ND[6] = "nd:inward half sweep"
NAMES_ND[7] = "nd:outward + recover wait"
NAMES_ND[4] = "nd:sep terms (+chk)"
NAMES_ND[5] = "nd:sep barrier (+chk)"
NAMES_ND[8] = "nd:correction (+chk)"
NAMES_CR = list(NAMES[:15]) + ["cr:reduce b + barrier"]
NAMES_CR[3] = "iter:w,b,u,beta + barrier"
NAMES_CR[7] = "cr:odd stages + barrier"
NAMES_CR[12] = "iter:outward + barrier (+epilogue)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--N", type=int, default=16)
    ap.add_argument("--cr", action="store_true", help="label the buckets of the cyclic-reduction build")
    ap.add_argument("--ki", action="store_true", help="label the buckets of the explicit-inverse build (N = 16)")
    ap.add_argument("--nd", action="store_true", help="label the buckets of the nested-dissection build")
    ap.add_argument("--copies", type=int, default=-1,
                    help=">= 0: every instance a copy of this instance of the C2 batch (seed 2)")
    a = ap.parse_args()
    import torch
    import mpcq
    if a.copies >= 0:  # identical instances: per-phase cost alone (256) vs co-resident (512)
        src = mpcq.synth.make_batch(1024, a.N, gaits=("trot",), seed=2)
        b = {k: np.ascontiguousarray(np.repeat(src[k][a.copies:a.copies + 1], a.batch, axis=0))
             for k in ("xref", "fsteps")}
    else:
        b = mpcq.synth.make_batch(a.batch, a.N, gaits=("trot",), seed=2000)
    dev = torch.device("cuda", 0)
    xr = torch.from_numpy(b["xref"]).to(dev)
    fs = torch.from_numpy(b["fsteps"]).to(dev)
    f0 = torch.empty((a.batch, 12), dtype=torch.float64, device=dev)
    st = torch.empty(a.batch, dtype=torch.int32, device=dev)
    it = torch.empty(a.batch, dtype=torch.int32, device=dev)
    stamps = torch.zeros((a.batch, 16), dtype=torch.int64, device=dev)
    eng = mpcq.Engine(a.N)
    mpcq.lib().mpcq_debug_set_stamps(eng._h, C.c_void_p(stamps.data_ptr()))
    eng.solve_device(a.batch, xr.data_ptr(), fs.data_ptr(), f0.data_ptr(), st.data_ptr(), it.data_ptr())
    torch.cuda.synchronize()
    S = stamps.cpu().numpy().astype(np.float64)
    its = it.cpu().numpy()
    names = NAMES_CR if a.cr else (NAMES_KI if a.ki else (NAMES_ND if a.nd else NAMES))
    tot = S[:, :13].sum(axis=1) + S[:, 15]
    print(f"batch {a.batch} N={a.N}: iters median {np.median(its)} max {its.max()}; "
          f"kernel ms (event) {eng.last_kernel_ms()[1]:.2f}")
    print(f"cycles per instance: median {np.median(tot):.3e}; per iteration {np.median(tot / its):.0f}")
    for i, nm in enumerate(names):
        share = S[:, i] / tot
        per_it = S[:, i] / its
        print(f"  {nm:18s} share {np.median(share) * 100:6.2f}%   cycles/iter {np.median(per_it):9.0f}")
    eng.close()


if __name__ == "__main__":
    main()
