"""Pins the CPU oracle (oracle/cpk_oracle.c) before it is trusted as the checker.

1. The reference's own fixtures: c++/src/capnp/testdata/{binary,packed,segmented,segmented-packed,
   flat,packedflat} (copied verbatim into tests/golden/) and the KATs of
   serialize-packed-test.c++:203-220 / doc/encoding.md:310-337 (tests/golden/kats.json).
2. tests/golden/ref_vectors.npz: outputs of the real reference codec compiled from
   /root/reference (tools/make_golden.py), incl. truncated / corrupted streams.
3. Live fuzz against oracle/_ref/libcpk_ref.so when that build is present.
"""
import json
import os

import numpy as np
import pytest

import cases
import pyoracle as P

G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def oracle():
    return P.Oracle()


def _read(name):
    with open(os.path.join(G, name), "rb") as f:
        return f.read()


def test_kats(oracle):
    kats = json.load(open(os.path.join(G, "kats.json")))["cases"]
    assert len(kats) == 13
    for k in kats:
        u = bytes(k["unpacked"])
        p = bytes(k["packed"])
        w = np.frombuffer(u, "<u8") if u else np.zeros(0, "<u8")
        assert oracle.pack_chunk(w) == p
        st, got, pos = oracle.unpack_exact(p, len(w))
        assert st == P.OK and pos == len(p) and got.tobytes() == u
        assert oracle.unpacked_size(p) == (P.OK, len(w))
        st, pos = oracle.skip_words(p, len(w))
        assert st == P.OK and pos == len(p)


def test_reference_fixtures(oracle):
    binary, packed = _read("binary"), _read("packed")
    pk, st = oracle.pack_flat(P.words_of(binary))
    assert st == P.OK and pk == packed
    seg, segp = _read("segmented"), _read("segmented-packed")
    pk, st = oracle.pack_flat(P.words_of(seg))
    assert st == P.OK and pk == segp
    # hazard #1: the same 125-segment message packed as ONE chunk differs
    assert len(oracle.pack_chunk(P.words_of(seg))) == 1348 != len(segp)
    flat, pflat = _read("flat"), _read("packedflat")
    assert oracle.pack_chunk(P.words_of(flat)) == pflat
    st, w, used = oracle.read_message(packed)
    assert st == P.OK and w.tobytes() == binary and used == len(packed)
    st, w, used = oracle.read_message(segp)
    assert st == P.OK and w.tobytes() == seg and used == len(segp)
    assert oracle.unpacked_size(pflat) == (P.OK, len(flat) // 8)


def test_ref_vectors(oracle):
    v = np.load(os.path.join(G, "ref_vectors.npz"))

    def items(name):
        d, off = v[name], v[name + "_off"]
        return [d[off[i]:off[i + 1]] for i in range(len(off) - 1)]

    for w, p in zip(items("chunk_in"), items("chunk_out")):
        assert oracle.pack_chunk(w) == p.tobytes()
    for w, p in zip(items("msg_in"), items("msg_out")):
        pk, st = oracle.pack_flat(w)
        assert st == P.OK and pk == p.tobytes()
    for i, (b, w) in enumerate(zip(items("rd_in"), items("rd_words"))):
        st, got, used = oracle.read_message(b.tobytes(), int(v["rd_limit"][i]))
        assert st == v["rd_status"][i], (i, st, v["rd_status"][i])
        if st == P.OK:
            assert got.tobytes() == w.tobytes()
            assert used == v["rd_consumed"][i]
    for i, b in enumerate(items("sz_in")):
        st, w = oracle.unpacked_size(b.tobytes())
        assert st == v["sz_status"][i]
        if st == P.OK:
            assert w == v["sz_words"][i]


needs_ref = pytest.mark.skipif(not P.reference_available(), reason="oracle/_ref not built")


@needs_ref
def test_live_fuzz_vs_reference(oracle):
    ref = P.Reference()
    rng = np.random.default_rng(7)
    for trial in range(150):
        prof = ["mixed", "bytes", "text", "zeros"][trial % 4]
        w = cases.random_words(rng, int(rng.integers(0, 1500)), prof)
        assert oracle.pack_chunk(w) == ref.pack_chunk(w)
    for trial in range(60):
        nseg = int(rng.integers(1, 12))
        m = cases.flat_message(rng, nseg, rng.integers(0, 300, size=nseg),
                               ["mixed", "bytes", "text"][trial % 3])
        segs = P.split_flat(m)
        pr = ref.pack_segments(segs)
        assert oracle.pack_flat(m)[0] == pr
        assert ref.pack_segments(segs, unbuffered=True) == pr  # 8 KiB-buffer path, :466-475
        # reader: valid, truncated, corrupted
        for b in (pr, pr[: len(pr) // 2], pr[:-1]):
            a = oracle.read_message(b)
            r = ref.read_message(b)
            assert a[0] == r[0]
            if a[0] == P.OK:
                assert a[1].tobytes() == r[1].tobytes() and a[2] == r[2]
        bb = bytearray(pr)
        bb[int(rng.integers(0, len(bb)))] ^= 0xFF
        a, r = oracle.read_message(bytes(bb)), ref.read_message(bytes(bb))
        assert a[0] == r[0]
        # skip + exact unpack of the body (flat-packed path, capnp.c++:1066-1071)
        body = oracle.pack_chunk(m)
        for k in (len(m), len(m) - 1, len(m) + 1):
            if k < 0:
                continue
            (so_, po_), (sr_, pr_) = oracle.skip_words(body, k), ref.skip_words(body, k)
            assert so_ == sr_ and (so_ != P.OK or po_ == pr_)  # position is moot after a throw
            so, wo, po = oracle.unpack_exact(body, k)
            sr, wr, pr2 = ref.unpack_exact(body, k)
            assert so == sr
            if so == P.OK:
                assert wo.tobytes() == wr.tobytes() and po == pr2


@needs_ref
def test_batch_vs_reference(oracle):
    ref = P.Reference()
    rng = np.random.default_rng(11)
    words, off = cases.message_batch(rng, 40)
    po, oo, so = oracle.pack_batch(words, off)
    pr, orr = ref.pack_batch(words, off)
    assert po.tobytes() == pr.tobytes() and (oo == orr).all() and (so == 0).all()
    wo, wo_off, st = oracle.unpack_batch(po, oo, len(words))
    assert (st == 0).all() and wo.tobytes() == words.tobytes() and (wo_off == off).all()
    # ref_unpack_batch reads into scratch space, which holds the segments only (no table,
    # serialize.c++:251-262): compare against the batch with the tables stripped.
    wr, wr_off = ref.unpack_batch(pr, orr, len(words))
    segs = [np.concatenate(P.split_flat(words[off[i]:off[i + 1]]) or [np.zeros(0, "<u8")])
            for i in range(len(off) - 1)]
    assert wr.tobytes() == np.concatenate(segs).tobytes()


# serialize-test.c++:533-543 ("large segment counts are rejected -- even UINT_MAX";
# security-advisories/2026-03-12-0-segment-count-overflow.md): first word ff ff ff ff 00 00 00 00,
# packed as the record 0f ff ff ff ff.
UINT_MAX_SEGMENTS = bytes([0x0F, 0xFF, 0xFF, 0xFF, 0xFF])


def test_uint_max_segment_count(oracle):
    w = np.frombuffer(bytes([0xFF] * 4 + [0] * 4), "<u8")
    assert oracle.pack_chunk(w) == UINT_MAX_SEGMENTS
    st, _, _ = oracle.read_message(UINT_MAX_SEGMENTS)
    assert st == P.TOO_MANY_SEGMENTS
    if P.reference_available():
        ref = P.Reference()
        assert ref.pack_chunk(w) == UINT_MAX_SEGMENTS
        assert ref.read_message(UINT_MAX_SEGMENTS)[0] == P.TOO_MANY_SEGMENTS
        assert "too many segments" in ref.last_error()


def test_c1_addressbook_fixture(oracle):
    """Config C1: the addressbook sample's message (samples/addressbook.c++:47-76) and its
    packed form, both hash-pinned to the compiled sample; the oracle packs the
    one to the other and reads it back (addressbook.c++:79, PackedFdMessageReader)."""
    import hashlib

    msg, packed = _read("addressbook.bin"), _read("addressbook.packed")
    assert hashlib.sha256(msg).hexdigest().startswith("6734639c")
    assert hashlib.sha256(packed).hexdigest().startswith("6cb6a027")
    w = P.words_of(msg)
    got, st = oracle.pack_flat(w)
    assert st == P.OK and got == packed
    rs, rw, used = oracle.read_message(packed)
    assert rs == P.OK and used == len(packed) and rw.tobytes() == msg


@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5", "c5r0of8"])
def test_manifest_prefixes(oracle, name):
    """The oracle's host generator + packer reproduce the reference's hashes for the first
    messages of every bench configuration (tests/golden/manifest.json, tools/make_manifest.py)."""
    import hashlib

    c = json.load(open(os.path.join(G, "manifest.json")))["configs"][name]
    pre = c["prefix"]
    off = oracle.gen_offsets(pre["nmsgs"], nseg=c["nseg"], seg_words=c["seg_words"],
                             seed=c["seed"], first_msg=c["first_msg"], msg_stride=c["msg_stride"])
    w = oracle.gen_messages(c["profile"], off, nseg=c["nseg"], seed=c["seed"],
                            first_msg=c["first_msg"], msg_stride=c["msg_stride"])
    assert int(off[-1]) == pre["words"]
    assert hashlib.sha256(w).hexdigest() == pre["sha256_words"]
    packed, poff, st = oracle.pack_batch(w, off)
    assert (st == 0).all() and len(packed) == pre["packed_bytes"]
    assert hashlib.sha256(packed).hexdigest() == pre["sha256_packed"]
    assert hashlib.sha256(poff.astype("<u8")).hexdigest() == pre["sha256_out_off"]
