"""The batch exchange's device placement (include/cpk.h cpk_copy_ranges, used by
capnproto_amd.shard.gather_packed for round-robin shards): byte ranges at any alignment and
length, including empty ones, land exactly at their destinations and nothing else is written."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import capnproto_amd

    c = capnproto_amd.Codec(0)
    yield c
    c.close()


def test_copy_ranges_places_every_range(codec):
    import torch

    rng = np.random.default_rng(5)
    n = 3000
    lens = rng.integers(0, 300, n)
    big = rng.random(n) < 0.05  # some long ranges: the 16-byte body loop
    lens[big] = rng.integers(300, 20000, int(big.sum()))
    lens[::97] = 0
    src_total = int(lens.sum()) + 64
    src = torch.from_numpy(rng.integers(0, 256, src_total, dtype=np.uint8)).to(codec.device)
    # sources back to back with random gaps; destinations a random permutation of the ranges
    gaps = rng.integers(0, 5, n)
    src_off = np.cumsum(np.concatenate([[0], lens[:-1] + gaps[:-1]]))
    src_off = np.minimum(src_off, src_total - lens)
    perm = rng.permutation(n)
    dst_off = np.zeros(n, np.int64)
    dst_off[perm] = np.cumsum(np.concatenate([[3], lens[perm][:-1]]))
    dst_total = int(dst_off.max() + lens.max() + 16)
    dst = torch.full((dst_total,), 0xA5, dtype=torch.uint8, device=codec.device)
    t = lambda x: torch.from_numpy(np.asarray(x, np.int64)).to(codec.device)  # noqa: E731
    codec.copy_ranges(src, t(src_off), t(dst_off), t(lens), dst)
    codec.sync()
    got = dst.cpu().numpy()
    s = src.cpu().numpy()
    want = np.full(dst_total, 0xA5, np.uint8)
    for so, do, ln in zip(src_off, dst_off, lens):
        want[do:do + ln] = s[so:so + ln]
    assert np.array_equal(got, want)


def test_gather_placement_of_round_robin_shards(codec):
    """gather_packed's device placement on one process: the packed shards of a round-robin
    assignment, staged rank after rank, placed message by message at their global offsets,
    equal one pack of the whole batch (the multi-rank exchange around it runs in the gloo tests,
    tests/test_shard.py)."""
    import torch

    from capnproto_amd.shard import shard_messages

    world, n_global = 3, 200
    off, total = codec.gen_offsets(n_global, seed=9)
    words = codec.gen_messages("mixed", off, total, seed=9)
    whole, woff, _ = codec.pack_messages(words, off)
    codec.sync()
    staged, loffs, gids = [], [], []
    for r in range(world):
        first, stride, count = shard_messages(r, world, n_global, "round_robin")
        o, tot = codec.gen_offsets(count, seed=9, first_msg=first, msg_stride=stride)
        w = codec.gen_messages("mixed", o, tot, seed=9, first_msg=first, msg_stride=stride)
        p, po, st = codec.pack_messages(w, o)
        codec.sync()
        assert (st == 0).all()
        staged.append(p[: int(po[-1].item())].clone())
        loffs.append(po.clone())
        gids.append(first + stride * torch.arange(count, device=codec.device))
    bases = np.cumsum([0] + [int(x.numel()) for x in staged])
    buf = torch.cat(staged)
    gid = torch.cat(gids)
    src = torch.cat([loffs[r][:-1] + int(bases[r]) for r in range(world)])
    size = torch.cat([loffs[r][1:] - loffs[r][:-1] for r in range(world)])
    gsize = torch.zeros(n_global, dtype=torch.int64, device=codec.device)
    gsize[gid] = size
    goff = torch.zeros(n_global + 1, dtype=torch.int64, device=codec.device)
    torch.cumsum(gsize, 0, out=goff[1:])
    out = torch.empty(int(goff[-1].item()), dtype=torch.uint8, device=codec.device)
    codec.copy_ranges(buf, src, goff[gid], size, out)
    codec.sync()
    P = int(woff[-1].item())
    assert torch.equal(goff, woff) and torch.equal(out, whole[:P])


class _OneProcessDist:
    """torch.distributed's calls as gather_packed makes them, for `world` simulated ranks whose
    packed shards live in this process: rank `rank` is the destination, the others' sends are
    the copies out of their tensors (the device branch of gather_packed runs for real)."""

    class P2POp:
        def __init__(self, op, tensor, peer):
            self.op, self.tensor, self.peer = op, tensor, peer

    def __init__(self, shards, rank=0):
        self.shards, self.rank = shards, rank  # shards[r] = (packed[:P], offsets[:n + 1], first, stride)

    def get_world_size(self):
        return len(self.shards)

    def get_rank(self):
        return self.rank

    def all_gather(self, parts, meta):
        import torch

        for r, (p, o, first, stride) in enumerate(self.shards):
            n = int(o.numel()) - 1
            parts[r].copy_(torch.tensor([int(p.numel()), n, first, stride, 0], dtype=torch.int64))

    def isend(self, *a):  # (never called on the destination)
        raise AssertionError("send on the destination rank")

    def irecv(self, *a):
        pass

    def batch_isend_irecv(self, ops):
        class Done:
            def wait(self):
                return True

        # rank r sends its bytes first, then its offsets (gather_packed's order)
        seen = {}
        for op in ops:
            assert op.op == self.irecv
            k = seen.get(op.peer, 0)
            p, o, _, _ = self.shards[op.peer]
            op.tensor.copy_(p if k == 0 else o[:-1])
            seen[op.peer] = k + 1
        return [Done() for _ in ops]


def test_gather_packed_device_branch(codec):
    """gather_packed itself (shard.py) on device tensors of round-robin shards: the all-gather
    of the ranks' metadata, the receives into the staging buffer, the global message ids and
    their checks, and the device placement by copy_ranges -- with the other ranks simulated in
    this process.  The result equals one pack of the whole batch; without codec= it refuses
    before any exchange."""
    import torch

    from capnproto_amd.shard import gather_packed, shard_messages

    world, n_global = 3, 151
    off, total = codec.gen_offsets(n_global, seed=13)
    words = codec.gen_messages("mixed", off, total, seed=13)
    whole, woff, _ = codec.pack_messages(words, off)
    codec.sync()
    shards = []
    for r in range(world):
        first, stride, count = shard_messages(r, world, n_global, "round_robin")
        o, tot = codec.gen_offsets(count, seed=13, first_msg=first, msg_stride=stride)
        w = codec.gen_messages("mixed", o, tot, seed=13, first_msg=first, msg_stride=stride)
        p, po, st = codec.pack_messages(w, o)
        codec.sync()
        assert (st == 0).all()
        shards.append((p[: int(po[-1].item())].clone(), po.clone(), first, stride))
    dist = _OneProcessDist(shards)
    p0, o0, first0, stride0 = shards[0]
    n0 = int(o0.numel()) - 1
    out, goff = gather_packed(p0, o0, n0, dst=0, dist=dist, device="cpu", first_msg=first0,
                              msg_stride=stride0, codec=codec)
    codec.sync()
    P = int(woff[-1].item())
    assert torch.equal(goff, woff) and torch.equal(out, whole[:P])
    with pytest.raises(ValueError, match="codec"):
        gather_packed(p0, o0, n0, dst=0, dist=dist, device="cpu", first_msg=first0,
                      msg_stride=stride0)
