"""GPU: the N>1 path (mpcq/shard.py) with the HIP engine in every rank.

Two ranks share the box's one MI355X (one process per rank, as bench.py runs one
per GPU; gloo carries the gather here because RCCL refuses two ranks on one
device).  Each rank solves its contiguous shard of the seeded C5-mix batch
through the C ABI; the gathered forces and statuses must equal one process's
solve of the whole batch bit for bit (instances are independent workgroups, so
neither the shard boundaries nor the batch size may change a result), and that
solve must match the oracle.  The CPU twin is tests/test_shard.py."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOTAL = 333  # uneven shards (167 + 166)


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
    import mpcq
    from mpcq import shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        b = shard.shard_batch(total, world, rank, 16, ("trot", "bound", "pace"), seed=11)
        with mpcq.Engine(16) as e:
            r = e.solve(b["xref"], b["fsteps"], 0, want_x=False)
        f0 = shard.gather_rows(dist, torch.from_numpy(r["f0"]), total, world, rank)
        st = shard.gather_rows(dist, torch.from_numpy(r["status"].astype(np.int64)), total, world, rank)
        it = shard.gather_rows(dist, torch.from_numpy(r["iters"].astype(np.int64)), total, world, rank)
        if rank == 0:
            np.savez(out, f0=f0.numpy(), status=st.numpy(), iters=it.numpy())
    finally:
        dist.destroy_process_group()


def test_two_ranks_engine_shards_match_single_process(tmp_path, oracle):
    import torch.multiprocessing as mp
    import mpcq
    out = str(tmp_path / "r0.npz")
    import time
    ctx = mp.spawn(_worker, args=(2, _free_port(), TOTAL, out), nprocs=2, join=False)
    deadline = time.monotonic() + 100  # a blocked rank (rendezvous, gather) fails the test, not the suite
    done = False
    while not done and time.monotonic() < deadline:
        done = ctx.join(timeout=5)
    if not done:
        for proc in ctx.processes:
            if proc.is_alive():
                proc.terminate()
        for proc in ctx.processes:
            proc.join(timeout=10)
        pytest.fail(f"ranks did not finish in time; exit codes {[proc.exitcode for proc in ctx.processes]}")
    got = np.load(out)
    g = mpcq.synth.make_batch(TOTAL, 16, gaits=("trot", "bound", "pace"), seed=11)
    with mpcq.Engine(16) as e:
        whole = e.solve(g["xref"], g["fsteps"], 0, want_x=False)
    assert np.array_equal(got["f0"], whole["f0"])
    assert np.array_equal(got["status"], whole["status"].astype(np.int64))
    assert np.array_equal(got["iters"], whole["iters"].astype(np.int64))
    ref = oracle.solve_batch(g["xref"], g["fsteps"], 0, nthreads=8)
    assert np.array_equal(whole["status"], ref["status"])
    assert np.array_equal(whole["iters"], ref["iters"])
    assert float(np.abs(whole["f0"] - ref["f0"]).max()) <= 1e-9
