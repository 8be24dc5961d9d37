"""Seeded input generators shared by the oracle and GPU parity tests.

The shapes target the packed codec's run rules (serialize-packed.c++:352-426): zero runs around
the 255/256-word cap, raw runs of words with exactly one zero byte (the `c >= 2` test at :403),
0xff words followed by 0xff words, chunk ends inside runs, and message framing with 1..N segments
(serialize.c++:311-357).
"""
from __future__ import annotations

import numpy as np


def word_with_zero_bytes(rng, n, zeros):
    """n words with exactly `zeros` zero bytes each (positions random)."""
    b = rng.integers(1, 256, size=(n, 8), dtype=np.uint8)
    for i in range(n):
        idx = rng.choice(8, size=zeros, replace=False)
        b[i, idx] = 0
    return b.reshape(-1).view("<u8").copy()


def random_words(rng, n, profile="mixed"):
    """Word arrays with controllable zero/raw structure."""
    if n == 0:
        return np.zeros(0, "<u8")
    if profile == "bytes":  # i.i.d. bytes, 60 % zero
        b = rng.integers(1, 256, size=n * 8, dtype=np.uint8)
        b[rng.random(n * 8) < 0.6] = 0
        return b.view("<u8").copy()
    if profile == "text":  # no zero bytes at all -> one long raw run family
        b = rng.integers(0x20, 0x7F, size=n * 8, dtype=np.uint8)
        return b.view("<u8").copy()
    if profile == "zeros":
        return np.zeros(n, "<u8")
    if profile == "locked":
        # one non-zero byte per word, itself a power of two: every record is 2 bytes and every
        # data byte, read as a tag, is a 2-byte record too -- the chains through the odd and the
        # even bytes never meet (parity-locked packed data)
        b = np.zeros((n, 8), np.uint8)
        b[np.arange(n), rng.integers(0, 8, size=n)] = (1 << rng.integers(0, 8, size=n)).astype(np.uint8)
        return b.reshape(-1).view("<u8").copy()
    # "mixed": a run-length mixture of every word class.
    out = np.zeros(n, "<u8")
    i = 0
    while i < n:
        kind = rng.integers(0, 6)
        length = int(rng.choice([1, 2, 3, 7, 63, 64, 65, 200, 254, 255, 256, 257, 300, 511, 513]))
        length = min(length, n - i)
        if kind == 0:
            pass  # zero words
        elif kind == 1:  # F words (no zero byte)
            out[i : i + length] = word_with_zero_bytes(rng, length, 0)
        elif kind == 2:  # R' words (exactly one zero byte)
            out[i : i + length] = word_with_zero_bytes(rng, length, 1)
        elif kind == 3:  # raw-eligible mixture of F and R'
            z = rng.integers(0, 2, size=length)
            for j in range(length):
                out[i + j] = word_with_zero_bytes(rng, 1, int(z[j]))[0]
        elif kind == 4:  # struct-like words with >= 2 zero bytes
            zz = rng.integers(2, 8, size=length)
            for j in range(length):
                out[i + j] = word_with_zero_bytes(rng, 1, int(zz[j]))[0]
        else:  # i.i.d. bytes
            out[i : i + length] = random_words(rng, length, "bytes")
        i += length
    return out


def edge_chunks():
    """Hand-made chunks around every run boundary the greedy packer has."""
    F = np.frombuffer(bytes(range(1, 9)), "<u8")[0]
    R1 = np.frombuffer(bytes([1, 2, 3, 0, 5, 6, 7, 8]), "<u8")[0]
    O2 = np.frombuffer(bytes([1, 0, 3, 0, 5, 6, 7, 8]), "<u8")[0]
    Z = np.uint64(0)
    cases = []
    for n in (1, 2, 255, 256, 257, 258, 511, 512, 513, 767, 768, 769):
        cases.append(np.full(n, Z, "<u8"))
        cases.append(np.full(n, F, "<u8"))
        cases.append(np.concatenate([[F], np.full(n, R1, "<u8")]))
        cases.append(np.concatenate([[O2], np.full(n, Z, "<u8"), [O2]]))
        cases.append(np.concatenate([[R1, R1], np.full(n, F, "<u8"), [Z]]))
    cases.append(np.array([F, Z, F, Z, R1, F, R1, Z, Z, O2], "<u8"))
    return cases


def flat_message(rng, nseg, seg_words, profile="mixed"):
    """A flat serialized message (table + segments)."""
    segs = [random_words(rng, int(s), profile) for s in seg_words[:nseg]]
    tw = nseg // 2 + 1
    table = np.zeros(tw * 2, "<u4")
    table[0] = nseg - 1
    for i, s in enumerate(segs):
        table[i + 1] = len(s)
    return np.concatenate([table.view("<u8")] + segs)


def message_batch(rng, nmsgs, max_seg=5, max_words=700, profile="mixed"):
    """Random batch of flat messages laid out back to back; returns (words, msg_word_off)."""
    msgs = []
    for _ in range(nmsgs):
        nseg = int(rng.integers(1, max_seg + 1))
        sizes = rng.integers(0, max_words + 1, size=nseg)
        msgs.append(flat_message(rng, nseg, sizes, profile))
    off = np.zeros(nmsgs + 1, "<u8")
    off[1:] = np.cumsum([len(m) for m in msgs])
    words = np.concatenate(msgs) if msgs else np.zeros(0, "<u8")
    return words, off
