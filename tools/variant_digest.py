"""Digest of the engine's outputs on fixed batches, to compare a library variant with the
production library bit for bit (run once per MPCQ_LIB_VARIANT, compare the lines):

    python tools/variant_digest.py [--N 16 32]

A variant that only changes instruction scheduling (mpc-tsid_amd/csrc/asmpass/nop_elide.py) must print the
same digests as the library it came from."""
import argparse
import hashlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, nargs="+", default=[16, 32])
    a = ap.parse_args()
    import mpcq
    for N in a.N:
        for name, over in (("default", {}), ("polish", dict(polish=2, polish_rounds=8, polish_refine_iter=10))):
            src = mpcq.synth.make_batch(1024 if N <= 16 else 512, N, gaits=("trot",), seed=2)
            with mpcq.Engine(N, **over) as e:
                out = e.solve(src["xref"], src["fsteps"], 0)
                h = hashlib.sha256()
                for k in sorted(out):
                    v = out[k]
                    if isinstance(v, np.ndarray):
                        h.update(k.encode())
                        h.update(np.ascontiguousarray(v).tobytes())
                print(f"N={N} {name}: iters {int(np.sum(out['iters']))} digest {h.hexdigest()[:16]}", flush=True)


if __name__ == "__main__":
    main()
