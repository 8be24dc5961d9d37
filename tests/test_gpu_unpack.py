"""GPU parity for UNPACK: libcpk_hip.so (through its C ABI) vs the CPU oracle.

Reference behaviour being matched: PackedMessageReader over an array (serialize-packed.c++:437-440
-> InputStreamMessageReader serialize.c++:202-302 -> PackedInputStream::tryRead :34-183), the
flat-packed read (capnp.c++:1066-1071) and computeUnpackedSizeInWords (:482-508).  Words are
compared bit-exactly for every message the reference accepts; statuses for every message.
"""
import os

import numpy as np
import pytest

import cases
import pyoracle as P
from gpu_util import concat_bytes, dev, host_u64

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


def gpu_unpack(codec, msgs, limit=None):
    """msgs: list of packed byte strings.  Returns (words per message or None, statuses)."""
    data, off = concat_bytes(msgs)
    cap = 300 + sum(130 * len(m) + 300 for m in msgs)
    words, woff, st = codec.unpack_messages(dev(codec, data), dev(codec, off), cap,
                                            nbytes=len(data), traversal_limit_words=limit)
    codec.sync()
    w = host_u64(words)
    woff = woff.cpu().numpy()
    st = st.cpu().numpy()
    out = [w[woff[i]:woff[i + 1]].copy() if st[i] == 0 else None for i in range(len(msgs))]
    return out, st, woff


def check_against_oracle(codec, oracle, msgs, limit=P.DEFAULT_TRAVERSAL_LIMIT):
    got, st, _ = gpu_unpack(codec, msgs, limit)
    for i, m in enumerate(msgs):
        rs, rw, used = oracle.read_message(m, limit, cap_words=300 + 260 * len(m))
        if rs == P.OK and used != len(m):
            rs = P.TRAILING_BYTES
        assert st[i] == rs, (i, st[i], rs, m[:40].hex())
        if rs == P.OK:
            assert got[i].tobytes() == rw.tobytes(), i


def test_reference_fixtures(codec):
    rd = lambda n: open(os.path.join(G, n), "rb").read()  # noqa: E731
    got, st, _ = gpu_unpack(codec, [rd("packed"), rd("segmented-packed"), rd("packed")])
    assert (st == 0).all()
    assert got[0].tobytes() == rd("binary") and got[2].tobytes() == rd("binary")
    assert got[1].tobytes() == rd("segmented")


@pytest.mark.parametrize("profile", ["mixed", "bytes", "text"])
def test_round_trip_batches(codec, oracle, profile):
    rng = np.random.default_rng(3 + len(profile))
    msgs = []
    for _ in range(150):
        nseg = int(rng.integers(1, 9))
        m = cases.flat_message(rng, nseg, rng.integers(0, 700, size=nseg), profile)
        msgs.append(oracle.pack_flat(m)[0])
    check_against_oracle(codec, oracle, msgs)


def test_large_messages_multi_tile(codec, oracle):
    """Messages spanning many 4 KiB tiles, incl. text (long raw runs) and long zero runs."""
    rng = np.random.default_rng(12)
    msgs = []
    for prof, n in (("mixed", 30000), ("text", 20000), ("zeros", 100000), ("bytes", 25000),
                    ("mixed", 9000)):
        m = cases.flat_message(rng, 3, [n // 3, n // 3, n // 3], prof)
        msgs.append(oracle.pack_flat(m)[0])
    check_against_oracle(codec, oracle, msgs)


def test_parity_locked_chains(codec, oracle):
    """Packed data whose record chains from odd and even bytes never meet, over many tiles and
    across message starts: the index kernel's capped merge walks hand such entries to the
    lane-parallel two-chain resolution (entry_chain), and resolve / expand must still follow the
    true chain."""
    rng = np.random.default_rng(31)
    msgs = []
    for n in (20000, 3000, 1, 2, 700, 16000, 5, 9000):
        parts = [cases.random_words(rng, n, "locked")]
        if n > 100:  # a lock that ends: ordinary data after it
            parts.append(cases.random_words(rng, 200, "mixed"))
            parts.append(cases.random_words(rng, n // 2, "locked"))
        w = np.concatenate(parts)
        m = np.concatenate([np.array([len(w) << 32], "<u8"), w])
        msgs.append(oracle.pack_flat(m)[0])
    check_against_oracle(codec, oracle, msgs)
    # small messages in front shift every lock against the 4 KiB tile grid
    for k in (1, 2, 3):
        tiny = oracle.pack_flat(cases.flat_message(rng, 1, [k], "mixed"))[0]
        check_against_oracle(codec, oracle, [tiny] + msgs[::-1])


def test_uint_max_segment_count(codec, oracle):
    """serialize-test.c++:533-543: a first word of ff ff ff ff 00 00 00 00 (segment count
    UINT_MAX + 1, packed 0f ff ff ff ff) is "Message has too many segments." -- alone, among
    valid messages, and inside a batch of many tiles (the split decode)."""
    bad = bytes([0x0F, 0xFF, 0xFF, 0xFF, 0xFF])
    assert oracle.pack_chunk(np.frombuffer(bytes([0xFF] * 4 + [0] * 4), "<u8")) == bad
    _, st, woff = gpu_unpack(codec, [bad])
    assert st[0] == P.TOO_MANY_SEGMENTS and woff[1] == woff[0]
    rng = np.random.default_rng(44)
    good = [oracle.pack_flat(cases.flat_message(rng, 2, [700, 900], "mixed"))[0] for _ in range(12)]
    msgs = good[:5] + [bad] + good[5:] + [bad]
    check_against_oracle(codec, oracle, msgs)
    _, st, _ = gpu_unpack(codec, msgs)
    assert list(np.nonzero(st)[0]) == [5, len(msgs) - 1]
    assert (st[[5, len(msgs) - 1]] == P.TOO_MANY_SEGMENTS).all()
    # the host entry point (its own staging path: one pinned buffer, one launch)
    import ctypes as C

    src = np.frombuffer(bad, np.uint8).copy()
    ioff = np.array([0, len(bad)], np.uint64)
    back = np.zeros(16, np.uint64)
    wo = np.zeros(2, np.uint64)
    st2 = np.full(1, -1, np.int32)
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    r = codec.lib.cpk_unpack_messages_host(codec.ctx, ptr(src), len(bad), ptr(ioff), 1, ptr(back),
                                           16, ptr(wo), ptr(st2), None)
    assert r == 0 and st2[0] == P.TOO_MANY_SEGMENTS and wo[1] == wo[0]


def test_error_cases(codec, oracle):
    rng = np.random.default_rng(21)
    msgs = []
    for _ in range(40):
        nseg = int(rng.integers(1, 6))
        m = cases.flat_message(rng, nseg, rng.integers(0, 300, size=nseg), "mixed")
        pk = oracle.pack_flat(m)[0]
        msgs.append(pk)
        msgs.append(pk[: int(rng.integers(0, len(pk)))])            # truncated
        bb = bytearray(pk)
        for _ in range(int(rng.integers(1, 4))):
            bb[int(rng.integers(0, len(bb)))] = int(rng.integers(0, 256))
        msgs.append(bytes(bb))                                       # corrupted
        msgs.append(pk + bytes([0x11, 0x22]))                        # trailing bytes
    msgs += [b"", b"\x00", b"\x00\x00", b"\x00\x01", bytes([0x0f, 0xff, 0x01, 0, 0]),
             bytes([0x03, 0xfe, 0x01]) + bytes(200), bytes([0xff]) + bytes(range(1, 9)) + b"\x05"]
    check_against_oracle(codec, oracle, msgs)


def test_traversal_limit(codec, oracle):
    rng = np.random.default_rng(4)
    msgs = [oracle.pack_flat(cases.flat_message(rng, 2, [100, 50], "mixed"))[0]
            for _ in range(10)]
    check_against_oracle(codec, oracle, msgs, limit=120)


def test_non_canonical_streams(codec, oracle):
    """The decoder must accept any valid stream (doc/encoding.md:323-329): raw runs holding
    zero bytes, non-maximal zero runs, runs split at arbitrary points."""
    rng = np.random.default_rng(8)
    msgs = []
    for _ in range(60):
        nwords = int(rng.integers(1, 400))
        body = bytearray()
        w = 0
        while w < nwords:
            k = int(rng.integers(0, 3))
            if k == 0:
                c = int(rng.integers(0, min(255, nwords - w - 1) + 1))
                body += bytes([0, c])
                w += 1 + c
            elif k == 1:
                c = int(rng.integers(0, min(255, nwords - w - 1) + 1))
                body += bytes([0xff]) + rng.integers(0, 256, 8 + 8 * c, dtype=np.uint8).tobytes()
                body.insert(len(body) - 8 * c, c)
                w += 1 + c
            else:
                tag = int(rng.integers(1, 255))
                body += bytes([tag]) + rng.integers(1, 256, bin(tag).count("1"),
                                                    dtype=np.uint8).tobytes()
                w += 1
        table = np.array([0, nwords], "<u4").tobytes()
        head = oracle.pack_chunk(np.frombuffer(table, "<u8"))
        msgs.append(head + bytes(body))
    check_against_oracle(codec, oracle, msgs)


def test_unpacked_size(codec, oracle):
    v = np.load(os.path.join(G, "ref_vectors.npz"))
    d, off = v["sz_in"], v["sz_in_off"]
    bufs = [d[off[i]:off[i + 1]].tobytes() for i in range(len(off) - 1)]
    rng = np.random.default_rng(1)
    bufs += [oracle.pack_chunk(cases.random_words(rng, int(n), "mixed"))
             for n in rng.integers(0, 5000, 20)]
    bufs += [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in (1, 2, 7, 33, 900)]
    bufs += [b"", bytes([5, 1]), bytes([0xff, 1, 2, 3, 4, 5, 6, 7, 8])]
    data, o = concat_bytes(bufs)
    sz, st = codec.unpacked_size(dev(codec, data), dev(codec, o), nbytes=len(data))
    codec.sync()
    sz, st = sz.cpu().numpy(), st.cpu().numpy()
    for i, b in enumerate(bufs):
        rs, rw = oracle.unpacked_size(b)
        assert st[i] == rs, (i, b[:20].hex())
        if rs == P.OK:
            assert sz[i] == rw, i


def test_unpack_chunks_flat_packed(codec, oracle):
    rng = np.random.default_rng(2)
    chunks = [cases.random_words(rng, int(n), p) for n, p in
              zip(rng.integers(0, 3000, 30), ["mixed", "text", "bytes", "zeros"] * 8)]
    bufs = [oracle.pack_chunk(c) for c in chunks]
    # error variants: expect one word more / less than encoded
    want = [len(c) for c in chunks]
    want[3] += 1
    want[5] = max(0, want[5] - 1)
    data, o = concat_bytes(bufs)
    woff = np.zeros(len(want) + 1, np.int64)
    woff[1:] = np.cumsum(want)
    words, st = codec.unpack_chunks(dev(codec, data), dev(codec, o), dev(codec, woff),
                                    nbytes=len(data))
    codec.sync()
    w, st = host_u64(words), st.cpu().numpy()
    for i, b in enumerate(bufs):
        rs, rw, pos = oracle.unpack_exact(b, want[i])
        if rs == P.OK and pos != len(b):
            rs = P.TRAILING_BYTES
        assert st[i] == rs, i
        if rs == P.OK:
            assert w[woff[i]:woff[i + 1]].tobytes() == rw.tobytes(), i


@pytest.mark.parametrize("profile", ["flat", "pointer", "text", "mixed"])
def test_device_round_trip_generated(codec, profile):
    """pack -> unpack on device reproduces the generated batch exactly (size-independent)."""
    import torch

    off, total = codec.gen_offsets(96, nseg=4, seg_words=2500, seed=3)
    words = codec.gen_messages(profile, off, total, nseg=4, seed=3)
    packed, moff, st = codec.pack_messages(words, off)
    nbytes = int(moff[-1].item())
    back, woff, st2 = codec.unpack_messages(packed, moff, total, nbytes=nbytes)
    codec.sync()
    assert (st2.cpu() == 0).all()
    assert torch.equal(woff, off)
    assert torch.equal(back[:total], words[:total])


@pytest.mark.parametrize("first,stride", [(0, 1), (3, 8)])
def test_c5_mixed_sizes_round_trip(codec, oracle, first, stride):
    """Config C5's shape (mixed profiles, 2^k-word messages, round-robin shard): device pack
    equals the oracle's bytes, device unpack restores every message."""
    import torch

    n = 6000
    off, total = codec.gen_offsets(n, nseg=1, seg_words=0, seed=11, first_msg=first,
                                   msg_stride=stride)
    words = codec.gen_messages("mixed", off, total, nseg=1, seed=11, first_msg=first,
                               msg_stride=stride)
    packed, moff, st = codec.pack_messages(words, off)
    codec.sync()
    P = int(moff[-1].item())
    ref, roff, rst = oracle.pack_batch(words.cpu().numpy().view(np.uint64),
                                       off.cpu().numpy().astype(np.uint64))
    assert (st.cpu().numpy() == 0).all()
    assert (moff.cpu().numpy() == roff.astype(np.int64)).all()
    assert packed[:P].cpu().numpy().tobytes() == ref.tobytes()
    back, woff, st2 = codec.unpack_messages(packed, moff, total, nbytes=P)
    codec.sync()
    s2 = st2.cpu().numpy()
    assert (s2 == 0).all(), np.nonzero(s2)[0][:10]
    assert torch.equal(woff, off)
    assert torch.equal(back[:total], words[:total])


def test_text_messages_many_tiles(codec, oracle):
    """Long raw-run streams: tiles whose first bytes sit inside raw data (fallback decoder)."""
    rng = np.random.default_rng(31)
    msgs = []
    for n in (512, 700, 1500, 2048, 4000, 9000):
        m = cases.flat_message(rng, 1, [n], "text")
        msgs.append(oracle.pack_flat(m)[0])
    check_against_oracle(codec, oracle, msgs)


def _raw_run_message(oracle, rng, p0, c, tail_words, nwords_delta=0, cut=None):
    """A packed message whose raw run record (0xff, 8 data bytes, count c, 8c raw bytes) starts at
    packed byte p0 of the message: 2-byte filler records before it, tail_words more after it.
    nwords_delta < 0 makes the segment table claim fewer words (the run then overshoots); cut
    truncates the packed bytes.  Returns the packed bytes."""
    body_words = lambda nfill: nfill + 1 + c + tail_words
    head = oracle.pack_chunk(np.array([0], "<u8"))  # placeholder size for the table word
    nfill = max(0, (p0 - len(head)) // 2)
    for _ in range(3):  # the table word's packed size depends on the word count
        nw = body_words(nfill) + nwords_delta
        head = oracle.pack_chunk(np.frombuffer(np.array([0, nw], "<u4").tobytes(), "<u8"))
        nfill = max(0, (p0 - len(head)) // 2)
    body = bytearray()
    for _ in range(nfill):
        body += bytes([0x01, int(rng.integers(1, 256))])
    if (p0 - len(head)) % 2:
        body[-2:] = bytes([0x03]) + rng.integers(1, 256, 2, dtype=np.uint8).tobytes()
    body += bytes([0xff]) + rng.integers(1, 256, 8, dtype=np.uint8).tobytes() + bytes([c])
    body += rng.integers(0, 256, 8 * c, dtype=np.uint8).tobytes()
    for _ in range(tail_words):
        body += bytes([0x01, int(rng.integers(1, 256))])
    m = head + bytes(body)
    return m[:cut] if cut is not None else m


def test_raw_runs_across_tiles(codec, oracle):
    """Raw runs crossing a 4 KiB tile boundary of the batch: the run's own tile writes the words
    staged with it, the next tile the rest from its own bytes (run_tail) -- except for a run that
    ends or breaks its message (its last record, a run overshooting the message's words, a
    message cut inside the run), whose tile writes it whole.  A valid message follows each case
    so that a stray write past a failing message shows; the next tile's guessed entry (the 64
    bytes before it are raw bytes) is wrong for most of them."""
    rng = np.random.default_rng(5)
    after = oracle.pack_flat(cases.flat_message(rng, 1, [300], "mixed"))[0]
    for p0 in (4090, 4080, 4070, 4050, 3900, 3000, 2100):
        for c in (1, 2, 5, 40, 255):
            batches = [
                [_raw_run_message(oracle, rng, p0, c, 20), after],        # run in the middle
                [_raw_run_message(oracle, rng, p0, c, 0), after],         # the message's last
                [_raw_run_message(oracle, rng, p0, c, 0, -1), after],     # overshoot
                [_raw_run_message(oracle, rng, p0, c, 10, -8), after],    # overshoot, then more
            ]
            full = _raw_run_message(oracle, rng, p0, c, 0)
            batches.append([full[: p0 + 10 + 4 * c], after])             # cut inside the run
            for msgs in batches:
                check_against_oracle(codec, oracle, msgs)
    # two tiles in a row each entered inside a run, runs of 255 words back to back
    for k in range(4):
        nw = 4 * 256
        body = bytearray()
        for _ in range(4):
            body += bytes([0xff]) + rng.integers(1, 256, 8, dtype=np.uint8).tobytes() + bytes([255])
            body += rng.integers(0, 256, 8 * 255, dtype=np.uint8).tobytes()
        head = oracle.pack_chunk(np.frombuffer(np.array([0, nw], "<u4").tobytes(), "<u8"))
        pad = oracle.pack_flat(cases.flat_message(rng, 1, [17 * k], "mixed"))[0]
        check_against_oracle(codec, oracle, [pad, head + bytes(body), after])


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 200, 256, 257])
def test_single_tile_batches(codec, oracle, n):
    """Batches of tiny messages that fit one 4 KiB tile: up to kUnpackFuseMsgs (256) messages the
    tile kernel reads the headers itself in the call's single launch (one thread per message,
    the word offsets by one workgroup scan), above that the header launch runs.  One
    truncated message and one with a UINT_MAX segment count ride along (serialize.c++:214-221)."""
    rng = np.random.default_rng(1000 + n)
    msgs = [oracle.pack_flat(cases.flat_message(rng, 1, [int(rng.integers(0, 2))], "mixed"))[0]
            for _ in range(n)]
    if n >= 2:
        msgs[n // 2] = msgs[n // 2][:-1]  # truncated
    if n >= 64:
        msgs[n - 2] = bytes([0x0F, 0xFF, 0xFF, 0xFF, 0xFF])  # segment count UINT_MAX + 1
    assert sum(len(m) for m in msgs) <= 4096
    check_against_oracle(codec, oracle, msgs)
