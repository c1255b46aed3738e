"""GPU: sliced batch solves (mpcq_set_slice) change no result.

Beyond 16 stages a sliced solve suspends every instance still iterating at the first ADMM
segment end after `slice` iterations, saves its iterate (x, z, y of every lane, rho, the loop
counters) and resumes the suspended instances in a second launch, the farthest from convergence
first, to their end -- the formulation, the scaling and the factorisation at the saved rho
recomputed, which gives the same bits.  Every
output must be bit-identical to the unsliced solve's: forces, x, y, statuses, iteration counts,
rho, rho updates, the ADMM status (and polish's outcome in the polish = 2 instantiation).
Slice lengths below, at and off the check interval (25), warm starts, the class order, the QP
entry point, max_iter ending between checks, the beyond-32-stage layout (N = 48), and N = 16,
where slicing is compiled out."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = ("f0", "x", "y", "status", "iters", "rho", "rho_updates", "admm_status", "polish", "polish_rounds")


def _same(a, b, tag=""):
    for k in KEYS:
        if k in a and a[k] is not None:
            assert np.array_equal(a[k], b[k], equal_nan=True), (tag, k)


def _pair(N, syn, slices, solve_kw=None, order_by_class=False, **params):
    import mpcq
    kw = dict(want_x=True, want_y=True)
    kw.update(solve_kw or {})
    with mpcq.Engine(N, **params) as e0:
        ref = e0.solve(syn["xref"], syn["fsteps"], order_by_class=order_by_class, **kw)
    for q in slices:
        with mpcq.Engine(N, **params) as e1:
            e1.set_slice(q)
            for _ in range(2 if order_by_class else 1):  # (the class table learns on the first)
                got = e1.solve(syn["xref"], syn["fsteps"], order_by_class=order_by_class, **kw)
                _same(ref, got, f"N={N} slice={q}")
    return ref


@pytest.mark.parametrize("N", [32, 20])
def test_slices_change_no_result(N):
    from mpcq import synth
    syn = synth.make_batch(300, N, gaits=("trot",), seed=2)
    ref = _pair(N, syn, (7, 25, 100, 333, 800))
    assert np.isin(ref["status"], (1, 2)).all()
    assert ref["iters"].max() > 800 and (ref["rho_updates"] > 0).any()  # slices cross rho updates


def test_slices_polish_and_class_order():
    from mpcq import synth
    syn = synth.make_batch(240, 32, gaits=("trot", "bound", "pace"), seed=7)
    _pair(32, syn, (50, 400), polish=2)
    _pair(32, syn, (300,), order_by_class=True)


def test_slices_warm_start_and_max_iter():
    from mpcq import synth
    import mpcq
    syn = synth.make_batch(128, 32, gaits=("trot",), seed=4)
    with mpcq.Engine(32) as e:
        cold = e.solve(syn["xref"], syn["fsteps"], want_x=True, want_y=True)
    warm = dict(warm_x=cold["x"], warm_y=cold["y"], rho=cold["rho"])
    _pair(32, syn, (10, 60), solve_kw=warm)
    # max_iter between two checks: the last slice ends on max_iter, not on a check
    ref = _pair(32, syn, (40, 130), max_iter=313)
    assert (ref["iters"] == 313).any()


def test_slices_qp_entry_point():
    import mpcq
    from mpcq import synth
    syn = synth.make_batch(96, 32, gaits=("trot",), seed=5)
    with mpcq.Engine(32) as e0:
        qp = e0.formulate(syn["xref"], syn["fsteps"])
        ref = e0.qp_solve(qp["Ax"], qp["l"], qp["u"])
    with mpcq.Engine(32) as e1:
        e1.set_slice(75)
        _same(ref, e1.qp_solve(qp["Ax"], qp["l"], qp["u"]), "qp")


@pytest.mark.parametrize("N", [48, 64])
def test_slices_beyond_32_stages(N):
    """The global-workspace layouts: S^-1 / R^-1 Q in the workspace (N > 32), the F_k rows and
    the scaled constraint values too (N > 48 / 49), whose recomputation the resume relies on."""
    from mpcq import synth
    syn = synth.make_batch(48 if N == 48 else 24, N, gaits=("trot",), seed=3)
    _pair(N, syn, (150,))


def test_slice_is_a_no_op_at_16_stages():
    from mpcq import synth
    syn = synth.make_batch(200, 16, gaits=("trot",), seed=2)
    _pair(16, syn, (25,))


def test_slices_multi_chunk_compaction():
    """More instances than the compaction's 1024-thread workgroup: the suspended ones are ranked
    in chunks (the residual-key counting sort's running offsets) -- still every instance once."""
    from mpcq import synth
    syn = synth.make_batch(2100, 20, gaits=("trot", "bound"), seed=6)
    _pair(20, syn, (60,))
