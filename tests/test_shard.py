"""Multi-GPU path on the CPU: message shards (capnproto_amd/shard.py) and the bench's whole-job
reductions, with world_size-2 gloo process groups (no GPU).  The data path has no collective:
each rank packs / unpacks its own messages, and a message's packed bytes do not depend on which
rank packs it -- checked against the oracle."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from capnproto_amd.shard import balanced_ranges, global_offsets, reduce_step, shard_messages


@pytest.mark.parametrize("mode", ["block", "round_robin"])
@pytest.mark.parametrize("world,n", [(1, 10), (2, 10), (2, 11), (8, 4096), (8, 13), (3, 2)])
def test_shards_partition_the_batch(mode, world, n):
    seen = []
    for r in range(world):
        first, stride, count = shard_messages(r, world, n, mode)
        seen += [first + stride * i for i in range(count)]
    assert sorted(seen) == list(range(n))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_batch():
    """The global batch: 12 flat messages (table word + one segment) known to every rank."""
    rng = np.random.default_rng(7)
    sizes = rng.integers(1, 300, 12)
    msgs = []
    for s in sizes:
        body = rng.integers(0, 2**63, int(s), dtype=np.uint64)
        body[rng.random(int(s)) < 0.4] = 0
        msgs.append(np.concatenate([np.array([int(s) << 32], dtype=np.uint64), body]))
    return msgs


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pyoracle

        o = pyoracle.Oracle()
        msgs = _global_batch()
        first, stride, count = shard_messages(rank, world, len(msgs), "round_robin")
        mine = [msgs[first + stride * i] for i in range(count)]
        off = np.cumsum([0] + [len(m) for m in mine]).astype(np.uint64)
        packed, poff, st = o.pack_batch(np.concatenate(mine), off)
        per_msg = [bytes(packed[int(poff[i]):int(poff[i + 1])]) for i in range(count)]
        alone = [o.pack_flat(m)[0] for m in mine]
        same = per_msg == alone
        red = reduce_step(0.5 + rank, float(off[-1] * 8), float(poff[-1]), 1.0 + rank, 2.0,
                          same, dist=dist)
        base, gtotal = global_offsets(int(poff[-1]), dist=dist)
        q.put((rank, red, same, [first + stride * i for i in range(count)],
               (base, gtotal, bytes(packed))))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shards_and_reduction():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    ids = sorted(out[0][3] + out[1][3])
    assert ids == list(range(12))
    for rank, red, same, _, _ in out:
        assert same, "per-message packed bytes depend on the shard"
        assert red["dt_max"] == 1.5 and red["pack_ms"] == 2.0
        assert red["ok_all"]
    assert out[0][1]["unpacked_all"] == out[1][1]["unpacked_all"] > 0
    # global placement from the all-gathered per-rank totals: rank 1 starts where rank 0 ends,
    # and the concatenation is the packed stream of the whole batch in shard order (rank 0's
    # messages, then rank 1's), packed here on one rank
    (b0, t0, p0), (b1, t1, p1) = out[0][4], out[1][4]
    assert b0 == 0 and b1 == len(p0) and t0 == t1 == len(p0) + len(p1)
    import pyoracle

    msgs = _global_batch()
    order = out[0][3] + out[1][3]
    whole = [msgs[i] for i in order]
    off = np.cumsum([0] + [len(m) for m in whole]).astype(np.uint64)
    packed, poff, st = pyoracle.Oracle().pack_batch(np.concatenate(whole), off)
    assert p0 + p1 == bytes(packed[: int(poff[-1])])


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_balanced_ranges(world):
    rng = np.random.default_rng(world)
    sizes = 2 ** rng.integers(3, 12, 5000) + 1  # C5-like: 2^k words + table word
    off = np.concatenate([[0], np.cumsum(sizes)])
    parts = balanced_ranges(off, world)
    assert sum(c for _, c in parts) == len(sizes)
    assert [f for f, _ in parts] == list(np.cumsum([0] + [c for _, c in parts])[:-1])
    loads = [int(off[f + c] - off[f]) for f, c in parts]
    assert max(loads) - min(loads) <= 2 * int(sizes.max())


def _gather_worker(rank, world, port, dst, q, mode="block"):
    import torch
    import torch.distributed as dist

    from capnproto_amd.shard import gather_packed

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pyoracle

        msgs = _global_batch()
        first, stride, count = shard_messages(rank, world, len(msgs), mode)
        mine = [msgs[first + stride * i] for i in range(count)]
        off = np.cumsum([0] + [len(m) for m in mine]).astype(np.uint64)
        packed, poff, st = pyoracle.Oracle().pack_batch(
            np.concatenate(mine) if count else np.zeros(0, np.uint64), off)
        # the device buffer shape of Codec.pack_messages: capacity past P, int64 offsets
        buf = torch.zeros(int(poff[-1]) + 64, dtype=torch.uint8)
        buf[: int(poff[-1])] = torch.from_numpy(np.asarray(packed[: int(poff[-1])]).copy())
        moff = torch.from_numpy(poff.astype(np.int64))
        if mode == "block":  # (contiguous ranges in rank order: no ids needed)
            out, offs = gather_packed(buf, moff, count, dst=dst, dist=dist)
        else:
            out, offs = gather_packed(buf, moff, count, dst=dst, dist=dist, first_msg=first,
                                      msg_stride=stride)
        q.put((rank, None if out is None else (bytes(out.numpy()), offs.numpy().tolist())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["block", "round_robin"])
@pytest.mark.parametrize("world,dst", [(2, 0), (2, 1), (3, 1)])
def test_gloo_gather_packed_equals_single_rank_pack(world, dst, mode):
    """The batch case: block or round-robin shards (C5's assignment) packed on
    each rank, gathered onto rank `dst` -- the gathered stream holds message k at position k and
    the stream and message offsets equal a single rank packing the whole batch (the reference's
    readers take messages back to back from one stream, serialize-packed-test.c++:348-371)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, dst, q, mode))
             for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(out[r] is None for r in range(world) if r != dst)
    got, goff = out[dst]
    import pyoracle

    msgs = _global_batch()
    off = np.cumsum([0] + [len(m) for m in msgs]).astype(np.uint64)
    packed, poff, st = pyoracle.Oracle().pack_batch(np.concatenate(msgs), off)
    assert got == bytes(packed[: int(poff[-1])])
    assert goff == [int(x) for x in poff]
