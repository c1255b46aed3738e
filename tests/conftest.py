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
    """Fixtures at the other horizons (gen_golden.py horizons): {N: {field: array}}."""
    d = np.load(os.path.join(GOLDEN, "golden_horizons.npz"))
    out = {}
    for N in d["horizons"]:
        pre = f"n{int(N)}_"
        out[int(N)] = {k[len(pre):]: d[k] for k in d.files if k.startswith(pre)}
    return out
