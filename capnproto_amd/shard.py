"""Multi-GPU batch sharding for the packed codec (host logic, no GPU needed).

The path shards by message: every message is packed / unpacked independently (a packed message
never refers to another), so N ranks -- one process per GPU -- each own a disjoint set of
messages and there is no exchange on the data path.  The only collectives are the bench's
timing / byte-count reductions (``reduce_step``), which run once per measurement, not per step,
and -- for the batch case, where the outputs must land on one GPU --
``gather_packed``: one all-gather of per-rank totals, then every rank's packed bytes sent point to
point (RCCL send/recv over xGMI under the "nccl" backend) straight into their global offset in the
destination rank's buffer.

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


def balanced_ranges(msg_word_off, world: int):
    """Byte-balanced contiguous partition: cut the message sequence where the
    running unpacked size crosses r/world of the total, so every rank gets a contiguous range
    of messages whose byte count is within one message of total/world (round-robin on mixed
    sizes is only balanced on average).  msg_word_off: n+1 word offsets (numpy array or torch
    tensor).  Returns [(first_msg, count)] per rank."""
    import numpy as np

    off = np.asarray(msg_word_off.cpu() if hasattr(msg_word_off, "cpu") else msg_word_off,
                     dtype=np.int64)
    n = len(off) - 1
    total = int(off[-1])
    cuts = [0]
    for r in range(1, world):
        target = (total * r) // world
        # first message whose start is at or past the target share
        cuts.append(max(cuts[-1], min(n, int(np.searchsorted(off[:n], target, side="left")))))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1] - cuts[r]) for r in range(world)]


def global_offsets(local_packed_total: int, dist=None, device=None):
    """Global output placement of each rank's packed bytes in the batch case:
    ONE all-gather of the per-rank packed totals (one u64 per rank); rank r's bytes go at the
    sum of the totals of ranks < r.  Returns (base of this rank, global total)."""
    import torch

    t = torch.tensor([local_packed_total], dtype=torch.int64, device=device)
    if dist is None:
        return 0, int(local_packed_total)
    parts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    vals = [int(p.item()) for p in parts]
    r = dist.get_rank()
    return sum(vals[:r]), sum(vals)


def gather_packed(packed, msg_out_off, nmsgs: int, dst: int = 0, dist=None, device=None,
                  first_msg=None, msg_stride: int = 1, codec=None):
    """The batch case of SURVEY.md 8(e): every rank's packed messages land on rank ``dst`` as ONE
    packed stream holding the global batch in global message order -- message k at position k,
    as one rank packing every message writes it and as the reference's readers take messages
    back to back from one stream (serialize-packed-test.c++:348-371) -- with the N_global + 1
    global byte offsets.

    packed: u8 tensor holding this rank's packed batch (at least P bytes); msg_out_off: its
    nmsgs + 1 int64 byte offsets (``Codec.pack_messages``).  Local message i is global message
    ``first_msg + msg_stride * i`` (``shard_messages``); first_msg None means the ranks hold
    contiguous ranges in rank order (block or byte-balanced shards).

    One all-gather of (P, nmsgs, first_msg, msg_stride) per rank, then each rank's packed bytes
    and local offsets sent point to point.  Contiguous ranges in rank order are received in
    place, at their global byte offsets (nothing copied after the receive but the rebasing of the
    offsets).  Otherwise (round-robin, C5) the bytes are received rank after rank into a staging
    buffer and every message is copied to its global offset -- the exclusive sum of the global
    per-message sizes -- by one device launch (``Codec.copy_ranges``, one wave per message; pass
    ``codec`` for device tensors; host tensors, as in the gloo tests, are copied by torch).

    Returns (stream, offsets) on ``dst`` and (None, None) on the other ranks."""
    import torch

    P = int(msg_out_off[nmsgs].item())
    if dist is None:
        return packed[:P], msg_out_off[: nmsgs + 1]
    if first_msg is not None and packed.device.type != "cpu" and codec is None:
        # (checked on every rank before any collective: the placement of non-contiguous shards on
        # the device needs the codec, and a rank failing after the exchange would strand the rest)
        raise ValueError("gather_packed: pass codec= to place device tensors of round-robin "
                         "shards (first_msg given)")
    world, rank = dist.get_world_size(), dist.get_rank()
    contiguous_flag = 1 if first_msg is None else 0
    meta = torch.tensor([P, nmsgs, 0 if first_msg is None else first_msg, msg_stride,
                         contiguous_flag], dtype=torch.int64, device=device)
    parts = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(parts, meta)
    sizes = [int(p[0].item()) for p in parts]
    counts = [int(p[1].item()) for p in parts]
    firsts = [int(p[2].item()) for p in parts]
    strides = [max(1, int(p[3].item())) for p in parts]
    bases = [sum(sizes[:r]) for r in range(world)]
    mbase = [sum(counts[:r]) for r in range(world)]
    # rank-order contiguous ranges: global message ids mbase[r] + i on every rank
    in_order = all(int(p[4].item()) == 1 or (firsts[r] == mbase[r] and (strides[r] == 1 or
                                                                      counts[r] <= 1))
                   for r, p in enumerate(parts))
    if rank != dst:
        ops = []
        if P:
            ops.append(dist.P2POp(dist.isend, packed[:P].contiguous(), dst))
        if nmsgs:
            ops.append(dist.P2POp(dist.isend, msg_out_off[:nmsgs].contiguous(), dst))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return None, None
    total, ntotal = sum(sizes), sum(counts)
    dev = packed.device
    # rank order: rank r's bytes at bases[r], its local offsets at mbase[r] -- the final layout
    # when the ranks hold contiguous ranges in rank order, else the staging of the placement
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    loff = torch.empty(ntotal + 1, dtype=torch.int64, device=dev)
    ops = []
    for r in range(world):
        if r == dst:
            continue
        if sizes[r]:
            ops.append(dist.P2POp(dist.irecv, buf[bases[r]:bases[r] + sizes[r]], r))
        if counts[r]:
            ops.append(dist.P2POp(dist.irecv, loff[mbase[r]:mbase[r] + counts[r]], r))
    reqs = dist.batch_isend_irecv(ops) if ops else []
    buf[bases[dst]:bases[dst] + P].copy_(packed[:P])
    loff[mbase[dst]:mbase[dst] + nmsgs].copy_(msg_out_off[:nmsgs])
    for req in reqs:
        req.wait()
    if in_order:
        for r in range(world):  # rank-local offsets -> global
            if counts[r] and bases[r]:
                loff[mbase[r]:mbase[r] + counts[r]] += bases[r]
        loff[ntotal] = total
        return buf, loff
    # global message id, size and source offset of every received message (rank order)
    gid = torch.cat([firsts[r] + strides[r] * torch.arange(counts[r], dtype=torch.int64,
                                                            device=dev)
                     for r in range(world)]) if ntotal else torch.zeros(0, dtype=torch.int64,
                                                                         device=dev)
    ends = loff[1:ntotal + 1].clone()
    for r in range(world):  # each rank's last message ends at its packed total
        if counts[r]:
            ends[mbase[r] + counts[r] - 1] = sizes[r]
    msize = ends - loff[:ntotal]
    src = loff[:ntotal] + torch.repeat_interleave(
        torch.tensor(bases, dtype=torch.int64, device=dev),
        torch.tensor(counts, dtype=torch.int64, device=dev))
    if ntotal and (int(gid.min().item()) < 0 or int(gid.max().item()) >= ntotal or
                   int(torch.bincount(gid, minlength=ntotal).max().item()) != 1):
        raise ValueError("gather_packed: the ranks' messages are not a permutation of the "
                         "global batch (first_msg / msg_stride)")
    gsize = torch.zeros(ntotal, dtype=torch.int64, device=dev)
    gsize[gid] = msize
    goff = torch.zeros(ntotal + 1, dtype=torch.int64, device=dev)
    torch.cumsum(gsize, 0, out=goff[1:])
    dst_off = goff[gid]
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    if dev.type == "cpu":
        # host tensors (the gloo tests): the same placement, message by message
        for s_, d_, n_ in zip(src.tolist(), dst_off.tolist(), msize.tolist()):
            out[d_:d_ + n_] = buf[s_:s_ + n_]
    else:
        codec.copy_ranges(buf, src, dst_off, msize, out)
    return out, goff


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
