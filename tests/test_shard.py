"""CPU: the N>1 path (instance sharding, mpcq/shard.py) with world_size 2 over
gloo -- the same helpers bench.py runs over RCCL.  Each rank solves its shard
(oracle stands in for the device) and the gathered forces must equal the
single-process solve of the whole batch, bit for bit."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import conftest  # noqa: F401  (paths)
    import torch
    import torch.distributed as dist
    from mpcq import shard
    from oracle import oracle as O
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        b = shard.shard_batch(total, world, rank, 16, ("trot", "bound", "pace"), seed=11)
        lo, hi = shard.shard_bounds(total, world, rank)
        assert b["xref"].shape[0] == hi - lo
        r = O.solve_batch(b["xref"], b["fsteps"], 0, nthreads=1)
        f0 = shard.gather_rows(dist, torch.from_numpy(r["f0"]), total, world, rank)
        st = shard.gather_rows(dist, torch.from_numpy(r["status"].astype(np.int64)), total, world, rank)
        t = shard.max_over_ranks(dist, float(rank + 1), "cpu", world)
        if rank == 0:
            np.savez(out, f0=f0.numpy(), status=st.numpy(), tmax=t)
    finally:
        dist.destroy_process_group()


def test_bounds():
    from mpcq.shard import shard_bounds
    assert [shard_bounds(5, 2, r) for r in range(2)] == [(0, 3), (3, 5)]
    assert [shard_bounds(65536, 8, r)[1] - shard_bounds(65536, 8, r)[0] for r in range(8)] == [8192] * 8
    assert shard_bounds(2, 4, 3) == (2, 2)
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


@pytest.mark.parametrize("total", [5, 6])
def test_two_rank_gloo_shards_match_single_process(tmp_path, oracle, total):
    import torch.multiprocessing as mp
    from mpcq import synth
    out = str(tmp_path / "r0.npz")
    mp.spawn(_worker, args=(2, _free_port(), total, out), nprocs=2, join=True)
    got = np.load(out)
    g = synth.make_batch(total, 16, gaits=("trot", "bound", "pace"), seed=11)
    ref = oracle.solve_batch(g["xref"], g["fsteps"], 0, nthreads=1)
    assert np.array_equal(got["f0"], ref["f0"])
    assert np.array_equal(got["status"], ref["status"])
    assert float(got["tmax"]) == 2.0
