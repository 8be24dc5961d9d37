"""GPU parity for stream boundary discovery: cpk_split_packed_stream.

Reference behaviour being matched: constructing one PackedMessageReader after another on the
same packed stream (serialize-packed-test.c++:348-371; InputStreamMessageReader
serialize.c++:202-302 over PackedInputStream serialize-packed.c++:34-183).  The expected split
comes from the CPU oracle reading message after message from the front of the remaining bytes;
words, word offsets, packed byte offsets and the reason reading stopped must all agree.
"""
import os

import numpy as np
import pytest

import cases
import pyoracle as P
from gpu_util import dev, host_u64

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def codec():
    import capnproto_amd

    c = capnproto_amd.Codec(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def oracle():
    return P.Oracle()


def oracle_split(oracle, data: bytes, limit=P.DEFAULT_TRAVERSAL_LIMIT, max_msgs=1 << 30):
    """The reference's reader loop: one message after another from the front of the stream."""
    pos, woff, ioff, words = 0, [0], [0], []
    stop = P.OK
    while len(woff) - 1 < max_msgs:
        if pos == len(data):
            break
        rest = data[pos:]
        st, w, used = oracle.read_message(rest, limit, cap_words=300 + 8 * len(rest))
        if st == P.CAPACITY:  # a highly compressed message: read it again with room for it
            st, w, used = oracle.read_message(rest, limit, cap_words=300 + 130 * len(rest))
        if st != P.OK:
            stop = st
            break
        words.append(w)
        pos += used
        woff.append(woff[-1] + len(w))
        ioff.append(pos)
    flat = np.concatenate(words) if words else np.zeros(0, np.uint64)
    return flat, np.array(woff), np.array(ioff), stop


def gpu_split(codec, data: bytes, cap=None, max_msgs=None, limit=None):
    arr = np.frombuffer(data, np.uint8).copy() if data else np.zeros(0, np.uint8)
    if cap is None:
        cap = 300 + 130 * len(data)
    if max_msgs is None:
        max_msgs = len(data) // 2 + 2
    words, woff, ioff, st, n = codec.split_packed_stream(dev(codec, arr), cap, max_msgs,
                                                         nbytes=len(data),
                                                         traversal_limit_words=limit)
    codec.sync()
    n = int(n.item())
    woff = woff[:n + 1].cpu().numpy()
    return (host_u64(words)[:woff[-1]].copy(), woff, ioff[:n + 1].cpu().numpy(),
            int(st[n].item()), st[:n].cpu().numpy())


def check(codec, oracle, data, limit=P.DEFAULT_TRAVERSAL_LIMIT, max_msgs=None):
    ew, ewoff, eioff, estop = oracle_split(oracle, data, limit,
                                           max_msgs if max_msgs is not None else 1 << 30)
    gw, gwoff, gioff, gstop, gst = gpu_split(codec, data, max_msgs=max_msgs, limit=limit)
    assert len(gwoff) == len(ewoff), (len(gwoff) - 1, len(ewoff) - 1, gstop, estop)
    assert (gst == P.OK).all()
    assert gstop == estop, (gstop, estop)
    assert (gwoff == ewoff).all()
    assert (gioff == eioff).all()
    assert gw.tobytes() == ew.tobytes()
    return len(ewoff) - 1


def test_two_messages_from_one_stream(codec, oracle):
    """serialize-packed-test.c++:348-371 with the reference's own fixtures."""
    rd = lambda n: open(os.path.join(G, n), "rb").read()  # noqa: E731
    a, b = rd("packed"), rd("segmented-packed")
    gw, woff, ioff, stop, _ = gpu_split(codec, a + b)
    assert stop == P.OK and list(ioff) == [0, len(a), len(a) + len(b)]
    assert gw.tobytes() == rd("binary") + rd("segmented")
    assert list(woff) == [0, len(rd("binary")) // 8, (len(rd("binary")) + len(rd("segmented"))) // 8]
    assert check(codec, oracle, b + a + a + b) == 4


def test_empty_stream(codec, oracle):
    gw, woff, ioff, stop, _ = gpu_split(codec, b"")
    assert stop == P.OK and list(woff) == [0] and list(ioff) == [0]


@pytest.mark.parametrize("profile", ["mixed", "bytes", "text"])
def test_mixed_messages(codec, oracle, profile):
    rng = np.random.default_rng(11 + len(profile))
    msgs = []
    for _ in range(300):
        nseg = int(rng.integers(1, 12))
        m = cases.flat_message(rng, nseg, rng.integers(0, 500, size=nseg), profile)
        msgs.append(oracle.pack_flat(m)[0])
    assert check(codec, oracle, b"".join(msgs)) == 300


def test_uniform_stretches(codec, oracle):
    """Same-size single-segment messages (the 64-per-step path), broken by other sizes, empty
    segments and multi-segment messages."""
    rng = np.random.default_rng(5)
    msgs = []
    for block in range(12):
        size = int(rng.integers(0, 40)) if block % 3 else 0
        for _ in range(int(rng.integers(1, 200))):
            msgs.append(oracle.pack_flat(cases.flat_message(rng, 1, [size], "mixed"))[0])
        nseg = int(rng.integers(1, 5))
        msgs.append(oracle.pack_flat(cases.flat_message(rng, nseg, [size] * nseg, "bytes"))[0])
    data = b"".join(msgs)
    assert check(codec, oracle, data) == len(msgs)
    assert check(codec, oracle, data, max_msgs=len(msgs) // 2) == len(msgs) // 2
    assert check(codec, oracle, data, max_msgs=130) == 130


def test_truncated_streams(codec, oracle):
    rng = np.random.default_rng(8)
    msgs = [oracle.pack_flat(cases.flat_message(rng, int(n), rng.integers(0, 60, size=int(n)),
                                                p))[0]
            for n, p in zip(rng.integers(1, 6, size=12), ["mixed", "text", "bytes"] * 4)]
    data = b"".join(msgs)
    cuts = sorted(set(int(c) for c in rng.integers(1, len(data), size=40)) |
                  {1, 2, 9, 10, len(msgs[0]) - 1, len(msgs[0]) + 1, len(data) - 1})
    for cut in cuts:
        check(codec, oracle, data[:cut])


def test_reader_failures(codec, oracle):
    rng = np.random.default_rng(9)
    good = [oracle.pack_flat(cases.flat_message(rng, 2, [5, 7], "mixed"))[0] for _ in range(3)]
    # a header claiming 512 segments (serialize.c++:217)
    too_many = oracle.pack_chunk(np.array([511 | (1 << 32)], np.uint64))
    check(codec, oracle, b"".join(good) + too_many + good[0])
    # segment count UINT_MAX + 1 (serialize-test.c++:533-543): the first word ff ff ff ff 00 00 00 00
    uint_max = bytes([0x0F, 0xFF, 0xFF, 0xFF, 0xFF])
    check(codec, oracle, uint_max)
    check(codec, oracle, b"".join(good) + uint_max + good[0])
    # a message larger than the traversal limit (serialize.c++:235)
    big = oracle.pack_flat(cases.flat_message(rng, 1, [300], "mixed"))[0]
    check(codec, oracle, good[0] + big + good[1], limit=100)
    # a zero run that crosses the end of a message: table (1 seg of 1 word), then 00 01 -- the
    # run carries one word into what would be the next message (serialize-packed.c++:128-131)
    cross = bytes([0x10, 0x01, 0x00, 0x01])
    check(codec, oracle, good[0] + cross + good[1])
    # a zero run crossing the first word of a message (its first read is 8 bytes)
    check(codec, oracle, good[0] + bytes([0x00, 0x03]) + good[1])
    # a raw run whose count crosses the message end while its bytes are cut off
    raw = bytes([0x10, 0x01, 0xff, 1, 2, 3, 4, 5, 6, 7, 8, 0x05, 9, 9])
    check(codec, oracle, good[1] + raw)


def test_capacity(codec, oracle):
    rng = np.random.default_rng(10)
    msgs = [cases.flat_message(rng, 1, [100], "mixed") for _ in range(6)]
    data = b"".join(oracle.pack_flat(m)[0] for m in msgs)
    cap = 3 * len(msgs[0]) + 5
    gw, woff, ioff, stop, _ = gpu_split(codec, data, cap=cap)
    assert len(woff) == 4 and stop == P.CAPACITY
    assert gw.tobytes() == np.concatenate(msgs[:3]).tobytes()


def test_large_uniform_stream(codec, oracle):
    """4096 x 64 KiB messages (config C2's shape) in one stream: offsets against the oracle's
    packed lengths, words against the generator."""
    import torch

    n, seg = 4096, 8191
    off, total = codec.gen_offsets(n, 1, seg, seed=7)
    words = codec.gen_messages("flat", off, total, 1, seed=7)
    packed, poff, st = codec.pack_messages(words, off)
    codec.sync()
    nbytes = int(poff[-1].item())
    w2, woff, ioff, status, cnt = codec.split_packed_stream(packed, total + 16, n + 1,
                                                            nbytes=nbytes)
    codec.sync()
    assert int(cnt.item()) == n and int(status[n].item()) == P.OK
    assert torch.equal(woff[:n + 1], off) and torch.equal(ioff[:n + 1], poff)
    assert torch.equal(w2[:total], words[:total])


def _mixed_stream(codec, n, seed):
    """n messages of 2^k + 1 words (k in 3..11; C5's shape), mixed profiles, packed back to
    back: (words, word offsets, packed bytes, packed offsets, total words, packed length)."""
    off, total = codec.gen_offsets(n, seed=seed)
    words = codec.gen_messages("mixed", off, total, seed=seed)
    packed, poff, st = codec.pack_messages(words, off)
    codec.sync()
    assert (st == 0).all()
    return words, off, packed, poff, total, int(poff[-1].item())


def test_split_c5_shape_million_messages(codec):
    """1 Mi mixed-size messages (C5's shape: 2^k-word messages of three profiles) in one stream,
    split across many 1 Mi-word blocks: every message boundary, packed offset and word against
    the generator's layout (whose packed bytes are pinned to the reference elsewhere)."""
    import torch

    n = 1 << 20
    words, off, packed, poff, total, nbytes = _mixed_stream(codec, n, 11)
    w2, woff, ioff, status, cnt = codec.split_packed_stream(packed, total + 16, n + 1,
                                                            nbytes=nbytes)
    codec.sync()
    assert int(cnt.item()) == n and int(status[n].item()) == P.OK
    assert (status[:n] == 0).all()
    assert torch.equal(woff[:n + 1], off) and torch.equal(ioff[:n + 1], poff)
    assert torch.equal(w2[:total], words[:total])


def test_split_limit_and_cut_in_later_blocks(codec):
    """max_msgs ending deep in the stream, and a stream cut inside a message many blocks in: the
    split stops exactly where the reference's reader loop would."""
    import torch

    n = 1 << 16
    words, off, packed, poff, total, nbytes = _mixed_stream(codec, n, 12)
    m = 40000  # several blocks in
    w2, woff, ioff, status, cnt = codec.split_packed_stream(packed, total + 16, m, nbytes=nbytes)
    codec.sync()
    assert int(cnt.item()) == m and int(status[m].item()) == P.OK
    assert torch.equal(woff[:m + 1], off[:m + 1]) and torch.equal(ioff[:m + 1], poff[:m + 1])
    # cut 3 bytes into message m's packed bytes: m whole messages, then premature end of input
    cut = int(poff[m].item()) + 3
    w2, woff, ioff, status, cnt = codec.split_packed_stream(packed, total + 16, n + 1, nbytes=cut)
    codec.sync()
    assert int(cnt.item()) == m and int(status[m].item()) == P.PREMATURE_EOF
    assert torch.equal(woff[:m + 1], off[:m + 1]) and torch.equal(ioff[:m + 1], poff[:m + 1])
    mw = int(off[m].item())
    assert torch.equal(w2[:mw], words[:mw])


def test_split_map_generations(codec):
    """Back-to-back splits of different streams into one output extent: the record-head map is
    filled only when its layout changes, so each call's heads must count and the previous
    call's must not (generation-tagged entries) -- including a call after a cut stream and after
    a call of another extent, which refills the map."""
    import torch

    n = 1 << 14
    streams = [_mixed_stream(codec, n, seed) for seed in (21, 22, 23)]
    cap = max(s[4] for s in streams) + 16
    for k in (0, 1, 2, 0, 1):
        words, off, packed, poff, total, nbytes = streams[k]
        w2, woff, ioff, status, cnt = codec.split_packed_stream(packed, cap, n + 1, nbytes=nbytes)
        codec.sync()
        assert int(cnt.item()) == n and int(status[n].item()) == P.OK, k
        assert torch.equal(woff[:n + 1], off) and torch.equal(ioff[:n + 1], poff), k
        assert torch.equal(w2[:total], words[:total]), k
    # a cut stream, then another extent (the map refilled), then the first extent again
    words, off, packed, poff, total, nbytes = streams[2]
    m = n // 2
    cut = int(poff[m].item()) + 5
    w2, woff, ioff, status, cnt = codec.split_packed_stream(packed, cap, n + 1, nbytes=cut)
    codec.sync()
    assert int(cnt.item()) == m and int(status[m].item()) == P.PREMATURE_EOF
    for c in (cap + 4096, cap):
        words, off, packed, poff, total, nbytes = streams[1]
        w2, woff, ioff, status, cnt = codec.split_packed_stream(packed, c, n + 1, nbytes=nbytes)
        codec.sync()
        assert int(cnt.item()) == n and int(status[n].item()) == P.OK
        assert torch.equal(woff[:n + 1], off) and torch.equal(ioff[:n + 1], poff)
        assert torch.equal(w2[:total], words[:total])


def test_split_messages_longer_than_blocks(codec):
    """Messages of 150 Ki words, longer than the split's 64 Ki-word blocks, between runs of small
    ones: blocks a message passes over take the in-order pass's serial path between windows it
    resolves in parallel, and every boundary still matches the generator's layout."""
    import torch

    parts = []
    for i, (n, seg) in enumerate(((3000, 200), (24, 150000), (5000, 60), (9, 150000),
                                  (2000, 1000))):
        off, total = codec.gen_offsets(n, 1, seg, seed=31 + i)
        words = codec.gen_messages("mixed", off, total, 1, seed=31 + i)
        parts.append((off, total, words))
    offs, tot = [torch.zeros(1, dtype=torch.int64, device=codec.device)], 0
    for off, total, _ in parts:
        offs.append(off[1:] + tot)
        tot += total
    off = torch.cat(offs)
    words = torch.cat([w[:t] for _, t, w in parts])
    n = off.numel() - 1
    packed, poff, st = codec.pack_messages(words, off)
    codec.sync()
    assert (st == 0).all()
    nbytes = int(poff[-1].item())
    w2, woff, ioff, status, cnt = codec.split_packed_stream(packed, tot + 16, n + 1, nbytes=nbytes)
    codec.sync()
    assert int(cnt.item()) == n and int(status[n].item()) == P.OK
    assert torch.equal(woff[:n + 1], off) and torch.equal(ioff[:n + 1], poff)
    assert torch.equal(w2[:tot], words[:tot])


def test_split_guess_off_chain(codec, oracle):
    """Messages whose words look like segment tables (valid one-segment headers at record heads)
    everywhere, so the guesses of the blocks land off the chain: the resolve walks those blocks
    again and the split is still the reference reader loop's (message lengths and their packed
    lengths from the oracle)."""
    rng = np.random.default_rng(21)
    msgs = []
    for _ in range(400):
        nw = int(rng.integers(20000, 40000))
        body = np.zeros(nw, "<u8")
        # every other word a plausible one-segment header of a 1..8-word message
        body[::2] = (rng.integers(0, 8, (nw + 1) // 2).astype(np.uint64) << np.uint64(32))
        body[1::2] = rng.integers(1 << 40, 1 << 62, nw // 2, dtype=np.uint64)
        msgs.append(np.concatenate([np.array([nw << 32], "<u8"), body]))
    packs = [oracle.pack_flat(m)[0] for m in msgs]
    data = b"".join(packs)
    gw, gwoff, gioff, gstop, gst = gpu_split(codec, data, cap=sum(len(m) for m in msgs) + 16,
                                             max_msgs=len(msgs) + 1)
    assert gstop == P.OK and (gst == P.OK).all() and len(gwoff) == len(msgs) + 1
    assert (gwoff == np.cumsum([0] + [len(m) for m in msgs])).all()
    assert (gioff == np.cumsum([0] + [len(p) for p in packs])).all()
    assert gw.tobytes() == np.concatenate(msgs).tobytes()
