"""Shared test setup: import paths, the `gpu` marker, golden fixtures."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mpc-tsid_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_golden(N):
    return dict(np.load(os.path.join(GOLDEN, f"golden_n{N}.npz")))


@pytest.fixture(scope="session")
def golden16():
    return load_golden(16)


@pytest.fixture(scope="session")
def golden32():
    return load_golden(32)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def golden_h():
    """Fixtures at the other horizons (gen_golden.py horizons / horizons_r3):
    {N: {field: array}}."""
    out = {}
    for name in ("golden_horizons.npz", "golden_horizons_r3.npz", "golden_horizons_r4.npz"):
        d = np.load(os.path.join(GOLDEN, name))
        for N in d["horizons"]:
            pre = f"n{int(N)}_"
            out[int(N)] = {k[len(pre):]: d[k] for k in d.files if k.startswith(pre)}
    return out


# the horizons the fixtures cover besides 16 / 32: multiples of 4 up to 32, N = 48
# (round 2), and round 3's non-multiples of 4, odd N and the range up to 64
# and round 4's layout switch points 49 (13 waves) and 50 (constraint values in the workspace)
FIXTURE_HORIZONS = (4, 5, 6, 8, 10, 12, 13, 20, 24, 28, 33, 36, 40, 48, 49, 50, 57, 64)
