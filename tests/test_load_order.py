"""libmpcq.so and torch share one HIP runtime whatever the import order.

torch bundles libamdhip64 (soname libamdhip64.so.7, the same as /opt/rocm's);
mpcq/_lib.py loads the copy torch will use before libmpcq.so, so a controller
may import mpcq first (tools/diag_runtime.py shows the two-runtime failure the
preload prevents).  Each case runs in a fresh interpreter."""
import os
import subprocess
import sys

import pytest

from conftest import PKG, REPO

CHILD = r'''
import os, sys
sys.path.insert(0, {pkg!r})
import mpcq
mpcq.lib()                       # libmpcq.so loaded before torch is imported
import torch
maps = sorted({{l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}})
print("RUNTIMES", len(maps), maps[0] if maps else "")
print("TORCH_LIB", os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
if {gpu!r}:
    import numpy as np
    n = torch.cuda.device_count()
    t = torch.arange(4, dtype=torch.float64, device="cuda")
    with mpcq.Engine(16, device=0) as eng:
        b = mpcq.synth.make_batch(2, 16, seed=5)
        r = eng.solve(b["xref"], b["fsteps"], mpcq.MODE_UPDATE)
    print("GPU", n, float(t.sum().item()), r["status"].tolist())
'''


def _run(gpu: bool):
    env = dict(os.environ)
    r = subprocess.run([sys.executable, "-c", CHILD.format(pkg=PKG, gpu=gpu)], capture_output=True, text=True,
                       timeout=300, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = dict(line.split(" ", 1) for line in r.stdout.strip().splitlines())
    return out


def test_one_runtime_when_mpcq_is_imported_first():
    out = _run(False)
    n, path = out["RUNTIMES"].split(" ", 1)
    assert n == "1", out
    assert os.path.realpath(path) == os.path.realpath(out["TORCH_LIB"])


def test_loaded_library_is_the_one_make_builds():
    import mpcq
    assert os.path.basename(mpcq._lib.LIB_PATH) == "libmpcq.so"
    # the in-tree library is up to date with its sources (make -q: nothing to rebuild)
    r = subprocess.run(["make", "-q", "-C", mpcq._lib.CSRC], capture_output=True)
    assert r.returncode == 0, "libmpcq.so is older than its sources: run make -C mpc-tsid_amd/csrc"


@pytest.mark.gpu
def test_torch_sees_the_device_after_mpcq():
    out = _run(True)
    n, s, st = out["GPU"].split(" ", 2)
    assert int(n) >= 1 and float(s) == 6.0, out
    assert st == "[1, 1]", out
