"""GPU parity for PACK: libcpk_hip.so (through its C ABI) vs the CPU oracle, bit-exact.

Reference behaviour being matched: PackedOutputStream::write per piece
(serialize-packed.c++:307-431) under writeMessage's chunking (serialize.c++:332-357).
"""
import json
import os

import numpy as np
import pytest

import cases
import pyoracle as P
from gpu_util import dev, host_u8, offsets

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


def gpu_pack_chunks(codec, chunks):
    words = np.concatenate(chunks) if chunks else np.zeros(0, "<u8")
    off = offsets([len(c) for c in chunks])
    out, coff = codec.pack_chunks(dev(codec, words), dev(codec, off))
    codec.sync()
    coff = coff.cpu().numpy()
    data = host_u8(out)[: int(coff[-1])]
    return data.tobytes(), coff


def gpu_pack_messages(codec, words, off):
    out, moff, st = codec.pack_messages(dev(codec, words), dev(codec, off))
    codec.sync()
    moff = moff.cpu().numpy()
    return host_u8(out)[: int(moff[-1])].tobytes(), moff, st.cpu().numpy()


def test_kats(codec):
    kats = json.load(open(os.path.join(G, "kats.json")))["cases"]
    chunks = [np.frombuffer(bytes(k["unpacked"]), "<u8") if k["unpacked"] else np.zeros(0, "<u8")
              for k in kats]
    data, coff = gpu_pack_chunks(codec, chunks)
    for i, k in enumerate(kats):
        assert data[coff[i]:coff[i + 1]] == bytes(k["packed"]), i


def test_reference_fixtures(codec):
    rd = lambda n: open(os.path.join(G, n), "rb").read()  # noqa: E731
    for src, dst in (("binary", "packed"), ("segmented", "segmented-packed")):
        w = P.words_of(rd(src))
        data, moff, st = gpu_pack_messages(codec, w, np.array([0, len(w)], np.int64))
        assert st[0] == P.OK and data == rd(dst) and moff[1] == len(rd(dst))
    flat = P.words_of(rd("flat"))
    data, _ = gpu_pack_chunks(codec, [flat])
    assert data == rd("packedflat")


def test_edge_chunks(codec, oracle):
    chunks = cases.edge_chunks()
    data, coff = gpu_pack_chunks(codec, chunks)
    for i, c in enumerate(chunks):
        assert data[coff[i]:coff[i + 1]] == oracle.pack_chunk(c), i


@pytest.mark.parametrize("profile", ["mixed", "bytes", "text", "zeros"])
def test_random_chunks(codec, oracle, profile):
    rng = np.random.default_rng(hash(profile) & 0xFFFF)
    lens = rng.integers(0, 3000, size=40)
    lens[::7] = 0  # empty chunks
    chunks = [cases.random_words(rng, int(n), profile) for n in lens]
    data, coff = gpu_pack_chunks(codec, chunks)
    ref = [oracle.pack_chunk(c) for c in chunks]
    assert (coff == offsets([len(r) for r in ref])).all()
    assert data == b"".join(ref)


def test_long_runs_across_tiles(codec, oracle):
    """Zero / raw / R' stretches much longer than a tile (2048 words) and a chunk boundary
    inside them; counts must see past the tile end."""
    F = np.frombuffer(bytes(range(1, 9)), "<u8")[0]
    R1 = np.frombuffer(bytes([1, 2, 0, 4, 5, 6, 7, 8]), "<u8")[0]
    chunks = [np.zeros(5000, "<u8"), np.full(3333, F, "<u8"),
              np.concatenate([np.full(700, R1, "<u8"), np.full(2000, F, "<u8")]),
              np.zeros(1023, "<u8"), np.zeros(1, "<u8"), np.full(1025, F, "<u8"),
              np.concatenate([[F], np.full(4000, R1, "<u8")])]
    for shift in (0, 1, 255, 511, 1000, 2047):  # move the structure against the tile grid
        cc = [np.zeros(shift, "<u8")] + chunks
        data, coff = gpu_pack_chunks(codec, cc)
        assert data == b"".join(oracle.pack_chunk(c) for c in cc), shift


@pytest.mark.parametrize("period", [512, 1024, 2048])
def test_runs_open_at_tile_end(codec, oracle, period):
    """A zero or raw stretch whose last head sits d words before a boundary at `period` (the
    pack kernel's wave: 512 words, workgroup tile: 2048) and that runs on e words past it, ended
    by an O word, a family change or a chunk start.  Across a tile boundary the count byte of
    the open run is written by the next tile."""
    F = np.frombuffer(bytes(range(1, 9)), "<u8")[0]
    O = np.frombuffer(bytes([1, 2, 0, 0, 5, 0, 0, 0]), "<u8")[0]
    R1 = np.frombuffer(bytes([1, 2, 0, 4, 5, 6, 7, 8]), "<u8")[0]
    chunks = []
    for fill in (0, F):
        for d in (1, 2, 17, 100, 255, 256, 257, 500):
            for e in (0, 1, 5, 200, 254, 255, 256, 300):
                for end in ("O", "fam", "chunk"):
                    head = np.full(period - d, O, "<u8")
                    run = np.full(d + e, fill, "<u8")
                    if end == "chunk":
                        chunks += [np.concatenate([head, run]), np.full(period - e, O, "<u8")]
                        continue
                    stop = R1 if (end == "fam" and fill == 0) else (np.uint64(0) if end == "fam"
                                                                     else O)
                    tail = np.full(period - e, O, "<u8")
                    tail[0] = stop
                    chunks.append(np.concatenate([head, run, tail]))
    data, coff = gpu_pack_chunks(codec, chunks)
    for i, c in enumerate(chunks):
        assert data[coff[i]:coff[i + 1]] == oracle.pack_chunk(c), i


@pytest.mark.parametrize("profile", ["mixed", "bytes", "text"])
def test_message_batches(codec, oracle, profile):
    rng = np.random.default_rng(99 + len(profile))
    words, off = cases.message_batch(rng, 120, max_seg=9, max_words=900, profile=profile)
    data, moff, st = gpu_pack_messages(codec, words, off.astype(np.int64))
    ref, roff, rst = oracle.pack_batch(words, off)
    assert (st == 0).all() and (moff == roff.astype(np.int64)).all()
    assert data == ref.tobytes()


def test_bad_framing(codec, oracle):
    rng = np.random.default_rng(5)
    words, off = cases.message_batch(rng, 30, max_seg=4, max_words=200)
    w = words.copy()
    # corrupt some tables: wrong sizes / absurd segment counts
    for k, m in enumerate(range(0, 30, 4)):
        t32 = w[off[m]:off[m] + 1].view("<u4")
        if k % 2:
            t32[1] += 1
        else:
            t32[0] = 0xFFFFFFFF
        w[off[m]] = t32.view("<u8")[0]
    data, moff, st = gpu_pack_messages(codec, w, off.astype(np.int64))
    ref, roff, rst = oracle.pack_batch(w, off)
    assert (st == rst).all() and (st[::4] == P.BAD_FRAMING).all()
    assert (moff == roff.astype(np.int64)).all() and data == ref.tobytes()


def test_generated_c2_sample(codec, oracle):
    """The bench workload (config C2 shape, 64 KiB flat-struct messages), 64 messages."""
    off, total = codec.gen_offsets(64, nseg=1, seg_words=8191, seed=1)
    words = codec.gen_messages("flat", off, total, nseg=1, seed=1)
    out, moff, st = codec.pack_messages(words, off)
    codec.sync()
    w = words.cpu().numpy().view(np.uint64)
    o = off.cpu().numpy()
    ref, roff, _ = oracle.pack_batch(w, o.astype(np.uint64))
    moff = moff.cpu().numpy()
    assert (moff == roff.astype(np.int64)).all()
    assert host_u8(out)[: int(moff[-1])].tobytes() == ref.tobytes()
    assert (st.cpu().numpy() == 0).all()


@pytest.mark.parametrize("profile", ["pointer", "text", "mixed"])
def test_generated_profiles(codec, oracle, profile):
    off, total = codec.gen_offsets(24, nseg=3, seg_words=3000, seed=7)
    words = codec.gen_messages(profile, off, total, nseg=3, seed=7)
    out, moff, st = codec.pack_messages(words, off)
    codec.sync()
    ref, roff, _ = oracle.pack_batch(words.cpu().numpy().view(np.uint64),
                                     off.cpu().numpy().astype(np.uint64))
    moff = moff.cpu().numpy()
    assert host_u8(out)[: int(moff[-1])].tobytes() == ref.tobytes()


def test_capacity_error(codec):
    import capnproto_amd
    import torch

    w = np.full(5000, np.frombuffer(bytes(range(1, 9)), "<u8")[0], "<u8")
    out = torch.empty(100, dtype=torch.uint8, device=codec.device)
    codec.pack_chunks(dev(codec, w), dev(codec, np.array([0, len(w)], np.int64)), out=out)
    with pytest.raises(capnproto_amd.CpkError) as ei:
        codec.sync()
    assert ei.value.status == capnproto_amd.CAPACITY


@pytest.mark.parametrize("profile", ["mixed", "bytes", "text"])
def test_pack_segments_device_list(codec, oracle, profile):
    """writePackedMessage(getSegmentsForOutput()) with every segment in its own device
    allocation (cpk_pack_segments: no host gather) -- bytes equal the oracle's."""
    import capnproto_amd

    rng = np.random.default_rng(21 + len(profile))
    for nseg in (1, 2, 3, 16, 130):
        sizes = rng.integers(0, 2500, size=nseg)
        sizes[rng.random(nseg) < 0.2] = 0
        segs = [cases.random_words(rng, int(s), profile) for s in sizes]
        tw = nseg // 2 + 1
        table = np.zeros(2 * tw, "<u4")
        table[0] = nseg - 1
        table[1:nseg + 1] = sizes
        flat = np.concatenate([table.view("<u8")] + [np.asarray(s, "<u8") for s in segs])
        want, st = oracle.pack_flat(flat)
        assert st == P.OK
        dsegs = [dev(codec, s) for s in segs]
        out, nb = codec.pack_segments(dsegs)
        codec.sync()
        n = int(nb.item())
        assert host_u8(out[:n]).tobytes() == want, (nseg, n, len(want))
    with pytest.raises(capnproto_amd.CpkError) as e:
        codec.pack_segments([])
    assert e.value.status == capnproto_amd.EMPTY_MESSAGE


def test_concurrent_contexts_two_streams(codec):
    """Two contexts pack and unpack full-size batches at the same time on two streams: the tile
    kernels only wait on lower tiles of their own launch (dispatched earlier), so neither can
    stall the other whatever else shares the GPU; statuses and bytes match a sequential run."""
    import capnproto_amd
    import torch

    other = capnproto_amd.Codec(0)
    try:
        jobs = []
        for seed, c in ((3, codec), (4, other)):
            off, total = c.gen_offsets(8192, seed=seed)  # C5-like sizes, ~45 MiB
            words = c.gen_messages("mixed", off, total, seed=seed)
            ref, rmoff, rst = c.pack_messages(words, off)
            c.sync()
            jobs.append((c, off, total, words, ref, rmoff, rst))
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        outs = []
        for (c, off, total, words, *_), s in zip(jobs, streams):
            with torch.cuda.stream(s):
                outs.append(c.pack_messages(words, off, stream=s))
        for (c, *_), s, (packed, moff, st) in zip(jobs, streams, outs):
            s.synchronize()
            c.sync(s)
        backs = []
        for (c, off, total, words, *_), s, (packed, moff, st) in zip(jobs, streams, outs):
            with torch.cuda.stream(s):
                backs.append(c.unpack_messages(packed, moff, total, stream=s))
        for s in streams:
            s.synchronize()
        for (c, off, total, words, ref, rmoff, rst), (packed, moff, st), (back, wo, ust) in zip(
                jobs, outs, backs):
            c.sync()
            P = int(rmoff[-1].item())
            assert int(moff[-1].item()) == P
            assert (st == 0).all() and (ust == 0).all()
            assert torch.equal(packed[:P], ref[:P]) and torch.equal(moff, rmoff)
            assert torch.equal(back[:total], words[:total]) and torch.equal(wo, off)
    finally:
        other.close()


def test_captured_then_eager_calls(codec):
    """A context whose previous call was captured into a HIP graph (on torch's capture stream)
    and whose next call comes eagerly on another stream: the cross-stream ordering event is
    skipped for a capturing stream, so neither the capture nor the eager call fails, and both
    give the sequential result (cpk_api.cpp order_streams)."""
    import torch

    off, total = codec.gen_offsets(64, seed=11)
    words = codec.gen_messages("mixed", off, total, seed=11)
    ref, rmoff, _ = codec.pack_messages(words, off)
    codec.sync()
    P = int(rmoff[-1].item())
    packed = torch.empty_like(ref)
    moff = torch.empty_like(rmoff)
    st = torch.empty(64, dtype=torch.int32, device=codec.device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        codec.pack_messages(words, off, out=packed, msg_out_off=moff, status=st)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        back, wo, ust = codec.unpack_messages(ref, rmoff, total, nbytes=P, stream=s)
    s.synchronize()
    codec.sync(s)
    g.replay()
    torch.cuda.synchronize()
    codec.sync()
    assert torch.equal(packed[:P], ref[:P]) and torch.equal(moff, rmoff) and (st == 0).all()
    assert torch.equal(back[:total], words[:total]) and (ust == 0).all()


@pytest.mark.gpu
def test_reserve_then_capture_fresh_context():
    """cpk_reserve on a fresh context makes every buffer a pack and an unpack of that size need
    (the scratch, the zero-at-rest chunk-start bitmap and header-scan descriptors), so both can be
    captured into a HIP graph as the first calls of the context (include/cpk.h cpk_reserve; no
    allocation or device synchronisation happens while the stream is capturing)."""
    import capnproto_amd
    import torch

    c = capnproto_amd.Codec(0)
    try:
        ref_codec = capnproto_amd.Codec(0)
        off, total = ref_codec.gen_offsets(300, seed=23)
        words = ref_codec.gen_messages("mixed", off, total, seed=23)
        ref, rmoff, _ = ref_codec.pack_messages(words, off)
        ref_codec.sync()
        P = int(rmoff[-1].item())
        ref_codec.close()
        c.reserve(total, P, 300)
        packed = torch.zeros_like(ref)
        moff = torch.zeros_like(rmoff)
        st = torch.full((300,), -1, dtype=torch.int32, device=c.device)
        back = torch.zeros(total + 8, dtype=torch.int64, device=c.device)
        woff = torch.zeros(301, dtype=torch.int64, device=c.device)
        ust = torch.full((300,), -1, dtype=torch.int32, device=c.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            c.pack_messages(words, off, out=packed, msg_out_off=moff, status=st)
            c.unpack_messages(ref, rmoff, total, nbytes=P, words=back, msg_word_off=woff,
                              status=ust)
        g.replay()
        torch.cuda.synchronize()
        c.sync()
        assert torch.equal(packed[:P], ref[:P]) and torch.equal(moff, rmoff) and (st == 0).all()
        assert torch.equal(back[:total], words[:total]) and torch.equal(woff, off)
        assert (ust == 0).all()
    finally:
        c.close()


@pytest.mark.parametrize("n", [1, 63, 64, 65, 200, 300])
def test_single_tile_batches(codec, oracle, n):
    """Batches of tiny messages within one 2048-word tile: the tile kernel frames the batch
    itself in the call's single launch (no framing or placement launch).  One message with a bad
    segment table rides along (writeMessage's framing, serialize.c++:311-357)."""
    rng = np.random.default_rng(2000 + n)
    words, off = cases.message_batch(rng, n, max_seg=2, max_words=2, profile="mixed")
    assert len(words) <= 2048
    if n >= 2:
        m = n // 2
        t32 = words[off[m]:off[m] + 1].view("<u4").copy()
        t32[1] += 1  # a segment size past the message
        words[off[m]] = t32.view("<u8")[0]
    data, moff, st = gpu_pack_messages(codec, words, off.astype(np.int64))
    ref, roff, rst = oracle.pack_batch(words, off)
    assert (st == rst).all() and (moff == roff.astype(np.int64)).all()
    assert data == ref.tobytes()
