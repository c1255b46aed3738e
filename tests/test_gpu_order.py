"""GPU: dispatch by gait class (MPCQ_FLAG_ORDER_BY_CLASS, mpcq_order.hip) changes no result.

A mixed-gait batch (trot / bound / pace interleaved, C5's generator) solved by one engine
without the flag and by another with it, three launches (the first learns the classes'
iteration counts, the later ones dispatch by them): every output -- forces, states,
statuses, iteration counts, info -- bit-identical.  Also a single-class batch and a batch
whose classes the table has not seen (unknown classes take the mean)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(eng, syn, flag):
    return eng.solve(syn["xref"], syn["fsteps"], want_x=True, want_y=True, order_by_class=flag)


def _same(a, b):
    for k in ("f0", "x", "y", "status", "iters", "rho", "rho_updates", "admm_status"):
        assert np.array_equal(a[k], b[k], equal_nan=True), k


@pytest.mark.parametrize("N", [16, 32])
def test_class_order_changes_no_result(N):
    import mpcq
    from mpcq import synth
    syn = synth.make_batch(600 if N == 16 else 300, N, gaits=("trot", "bound", "pace"), seed=7)
    with mpcq.Engine(N) as e0, mpcq.Engine(N) as e1:
        ref = _solve(e0, syn, False)
        assert np.isin(ref["status"], (1, 2)).all()
        for _ in range(3):
            _same(ref, _solve(e1, syn, True))
        # a single-class batch (identity order inside the class) and classes never seen
        one = synth.make_batch(200, N, gaits=("trot",), seed=8)
        _same(_solve(e0, one, False), _solve(e1, one, True))
        walk = synth.make_batch(130, N, gaits=("bound",), seed=9)
        with mpcq.Engine(N) as e2:
            _same(_solve(e0, walk, False), _solve(e2, walk, True))


def test_class_order_multi_chunk_batch():
    """B > 1024: the order kernel ranks the batch in chunks of its 1024-thread workgroup, each
    chunk's positions continuing the buckets' running offsets -- the dispatch must still be a
    permutation (every instance solved once: outputs equal to the unordered solve's)."""
    import mpcq
    from mpcq import synth
    syn = synth.make_batch(2600, 16, gaits=("trot", "bound", "pace"), seed=11)
    with mpcq.Engine(16) as e0, mpcq.Engine(16) as e1:
        ref = _solve(e0, syn, False)
        assert np.isin(ref["status"], (1, 2)).all()
        for _ in range(2):
            _same(ref, _solve(e1, syn, True))
