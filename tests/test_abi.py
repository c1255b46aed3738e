"""CPU: the C-ABI library (libmpcq.so) loads and exports every entry point
include/mpcq.h declares; host-side entry points that need no device agree with
the reference-generated fixtures.  No kernel is launched (no GPU here)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "mpcq.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return sorted(set(re.findall(r"\b(mpcq_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def mpcq():
    import mpcq as m
    m.build()
    return m


def test_exports_every_declared_symbol(mpcq):
    names = header_functions()
    assert len(names) >= 14
    lib = mpcq.lib()
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(mpcq._lib.EXPORTS)


def test_abi_version(mpcq):
    assert mpcq.lib().mpcq_abi_version() == 3


def test_default_params_match_reference(mpcq, golden16, oracle):
    p = mpcq.default_params()
    # MPC.py:28 mass, :35-37 gI (the full 3x3 that overwrites :31), :39 mu, :227-228 fz bound
    assert p.mass == 2.50000279
    assert np.array_equal(np.array(p.gI[:]).reshape(3, 3),
                          np.array([[3.09249e-2, -8.00101e-7, 1.865287e-5],
                                    [-8.00101e-7, 5.106100e-2, 1.245813e-4],
                                    [1.865287e-5, 1.245813e-4, 6.939757e-2]]))
    assert p.mu == 0.9 and p.fz_max == 25.0
    # cost diagonal of the reference formulation (captured into the fixture)
    Pd = np.concatenate([np.tile(np.array(p.state_weights[:]), 16), np.full(192, p.force_weight)])
    assert np.array_equal(Pd, golden16["P"])
    # OSQP 0.6 defaults + the reference's eps (MPC.py:414-416)
    assert (p.rho, p.sigma, p.alpha) == (0.1, 1e-6, 1.6)
    assert (p.eps_abs, p.eps_rel) == (1e-7, 1e-7)
    assert (p.max_iter, p.check_termination, p.scaling, p.polish) == (4000, 25, 10, 0)
    assert (p.eps_prim_inf, p.eps_dual_inf, p.dual_warm) == (1e-4, 1e-4, 0)
    # same constants as the oracle's restatement
    o = oracle.default_params()
    for name, _ in p._fields_:
        if name != "reserved":
            assert np.array_equal(np.ravel(getattr(p, name)), np.ravel(getattr(o, name))), name


@pytest.mark.parametrize("N", [16, 32])
def test_dims_and_pattern(mpcq, N, golden16, golden32):
    g = golden16 if N == 16 else golden32
    n, m, nnz = C.c_int32(), C.c_int32(), C.c_int32()
    assert mpcq.lib().mpcq_dims(N, C.byref(n), C.byref(m), C.byref(nnz)) == 0
    assert (n.value, m.value, nnz.value) == (24 * N, 44 * N, 126 * N - 18)
    indptr, indices = mpcq.pattern(N)
    assert np.array_equal(indptr, g["indptr"]) and np.array_equal(indices, g["indices"])


def test_supported_horizons(mpcq):
    assert mpcq.supported_horizons() == list(range(4, 65))


@pytest.mark.parametrize("N", [4, 5, 6, 8, 10, 12, 13, 20, 24, 28, 33, 36, 40, 48, 57, 64])
def test_pattern_other_horizons(mpcq, N, golden_h):
    indptr, indices = mpcq.pattern(N)
    assert np.array_equal(indptr, golden_h[N]["indptr"]) and np.array_equal(indices, golden_h[N]["indices"])


def test_errors_are_codes_not_crashes(mpcq):
    lib = mpcq.lib()
    h = C.c_void_p()
    p = mpcq.default_params()
    # unsupported horizon, then a device index no box has: both fail with a message, no abort
    assert lib.mpcq_create(0, 65, C.byref(p), C.byref(h)) != 0
    assert not h.value
    assert len(lib.mpcq_last_error()) > 0
    assert lib.mpcq_create(4096, 16, C.byref(p), C.byref(h)) != 0
    assert len(lib.mpcq_last_error()) > 0
    with pytest.raises(mpcq.MpcqError):
        mpcq.Engine(16, device=4096)
    # bad parameters are rejected before any device work
    bad = mpcq.default_params(alpha=2.5)
    assert lib.mpcq_create(0, 16, C.byref(bad), C.byref(h)) != 0
    for bad_pol in (dict(polish=3), dict(polish=1, delta=0.0), dict(polish=2, polish_rounds=0)):
        pol = mpcq.default_params(**bad_pol)
        assert lib.mpcq_create(0, 16, C.byref(pol), C.byref(h)) == -1, bad_pol
    lib.mpcq_destroy(None)  # destroying NULL returns a code, never crashes
