"""Instance sharding across ranks (one process per GPU).

Instances are independent QPs, so the batch is split into contiguous shards
with no data-path collective; the only collectives are the max-over-ranks
timing reduction and, optionally, a gather of the 12 forces per instance to
rank 0 (RCCL over xGMI on the GPU box, gloo in the CPU tests).
"""
from __future__ import annotations


def shard_bounds(total: int, world: int, rank: int):
    """Contiguous shard [lo, hi) of rank ``rank``: ceil(total / world) per rank, the last ones short."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    per = -(-int(total) // world)
    lo = min(rank * per, int(total))
    return lo, min(lo + per, int(total))


def shard_batch(total: int, world: int, rank: int, n_steps: int, gaits, seed: int):
    """This rank's slice of the seeded global synthetic batch (mpcq.synth.make_batch(total, ...)),
    generated alone: the batch is seeded per block of synth.CHUNK instances, so a rank
    builds only the blocks of its own shard."""
    from . import synth
    lo, hi = shard_bounds(total, world, rank)
    return synth.make_batch(total, n_steps, gaits=gaits, seed=seed, lo=lo, hi=hi)


def gather_rows(dist, t, total: int, world: int, rank: int):
    """all_gather a per-rank (rows, ...) tensor of uneven length into the (total, ...) global one
    (pads every shard to ceil(total / world) rows)."""
    import torch
    per = -(-int(total) // world)
    pad = torch.zeros((per,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    out = []
    for r in range(world):
        lo, hi = shard_bounds(total, world, r)
        out.append(parts[r][: hi - lo])
    return torch.cat(out)


def max_over_ranks(dist, value: float, device, world: int) -> float:
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if world > 1 or (dist.is_available() and dist.is_initialized()):
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
