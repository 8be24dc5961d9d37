"""Multi-GPU batch sharding for the packed codec (host logic, no GPU needed).

The path shards by message: every message is packed / unpacked independently (a packed message
never refers to another), so N ranks -- one process per GPU -- each own a disjoint set of
messages and there is no exchange on the data path.  The only collectives are the bench's
timing / byte-count reductions (``reduce_step``), which run once per measurement, not per step.

Two assignments of a global batch of ``n_global`` messages to ``world`` ranks:
  * ``block``       rank r owns messages [r*n_local, (r+1)*n_local)   (configs C2-C4)
  * ``round_robin`` rank r owns messages r, r+world, r+2*world, ...      (config C5)
Both give every rank the same count when world divides n_global.
"""
from __future__ import annotations


def shard_messages(rank: int, world: int, n_global: int, mode: str = "block"):
    """(first_msg, stride, count) of the messages rank `rank` owns: global ids
    first_msg + stride * i for i in [0, count)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    if mode == "block":
        base, extra = divmod(n_global, world)
        count = base + (1 if rank < extra else 0)
        first = rank * base + min(rank, extra)
        return first, 1, count
    if mode == "round_robin":
        count = (n_global - rank + world - 1) // world if n_global > rank else 0
        return rank, world, count
    raise ValueError(f"unknown shard mode {mode!r}")


def reduce_step(dt_s: float, unpacked: float, packed: float, pack_ms: float, unpack_ms: float,
                ok: bool, dist=None, device=None):
    """Whole-job numbers of one measurement: time = max over ranks (the job ends when the
    slowest rank ends), bytes = sum over ranks, kernel times = max, ok = all ranks bit-exact."""
    import torch

    t = torch.tensor([dt_s, unpacked, packed, pack_ms, unpack_ms], dtype=torch.float64,
                     device=device)
    o = torch.tensor([1 if ok else 0], dtype=torch.int64, device=device)
    if dist is None:
        tmax = tsum = t
    else:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        dist.all_reduce(o, op=dist.ReduceOp.MIN)
    return {
        "dt_max": float(tmax[0]),
        "unpacked_all": float(tsum[1]),
        "packed_all": float(tsum[2]),
        "pack_ms": float(tmax[3]),
        "unpack_ms": float(tmax[4]),
        "ok_all": bool(o.item()),
    }
