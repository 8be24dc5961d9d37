#!/usr/bin/env python3
"""Generate tests/golden/ref_vectors.npz from the REAL reference codec (oracle/_ref/libcpk_ref.so).

Run in the container that holds /root/reference after `make -f oracle/Makefile.ref`.  The vectors
are data: seeded inputs plus the reference's outputs (packed bytes, decoded words, status codes,
bytes consumed).  They pin oracle/cpk_oracle.c where the reference build is absent.

    python tools/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import cases  # noqa: E402
import pyoracle as P  # noqa: E402


def main():
    ref = P.Reference()
    rng = np.random.default_rng(20261015)
    chunk_in, chunk_out = [], []
    # a1: single chunks (PackedOutputStream::write) -- edge shapes + fuzz
    for c in cases.edge_chunks():
        chunk_in.append(c)
        chunk_out.append(np.frombuffer(ref.pack_chunk(c), np.uint8))
    for prof in ("mixed", "bytes", "text", "zeros"):
        for n in (0, 1, 5, 64, 300, 1000, 2100):
            c = cases.random_words(rng, n, prof)
            chunk_in.append(c)
            chunk_out.append(np.frombuffer(ref.pack_chunk(c), np.uint8))
    # a5/a7: whole messages (writePackedMessage) with 1..10 segments
    msg_in, msg_out = [], []
    for nseg in (1, 2, 3, 4, 7, 10, 33):
        for prof in ("mixed", "bytes", "text"):
            sizes = rng.integers(0, 400, size=nseg)
            m = cases.flat_message(rng, nseg, sizes, prof)
            msg_in.append(m)
            msg_out.append(np.frombuffer(ref.pack_segments(P.split_flat(m)), np.uint8))
    # a2/a8: reader over arbitrary (valid, truncated, corrupted) packed streams
    rd_in, rd_status, rd_words, rd_consumed, rd_limit = [], [], [], [], []

    def add_read(b, limit=P.DEFAULT_TRAVERSAL_LIMIT):
        st, w, used = ref.read_message(bytes(b), limit)
        rd_in.append(np.frombuffer(bytes(b), np.uint8))
        rd_status.append(st)
        rd_words.append(w)
        rd_consumed.append(used)
        rd_limit.append(limit)

    for m in msg_out[:9]:
        b = m.tobytes()
        add_read(b)
        for cut in sorted(set([0, 1, 2, 5, 9, len(b) // 2, len(b) - 1])):
            add_read(b[:cut])
        for _ in range(6):
            bb = bytearray(b)
            pos = int(rng.integers(0, len(bb)))
            bb[pos] = int(rng.integers(0, 256))
            add_read(bb)
        add_read(b, limit=3)
    for _ in range(40):
        add_read(rng.integers(0, 256, size=int(rng.integers(1, 60)), dtype=np.uint8).tobytes())
    add_read(bytes([0x0f, 0xff, 0x01, 0, 0]))            # 0x1ff = 511 -> 512 segments
    add_read(bytes([0x03, 0xfe, 0x01]) + bytes(200))      # 511 segments (allowed count)
    add_read(bytes([0x00, 0x00]))                         # empty single segment
    add_read(bytes([0x00, 0x01]))                         # run overshoot in first word
    # a4: computeUnpackedSizeInWords
    sz_in, sz_status, sz_words = [], [], []
    for m in msg_out[:6]:
        b = m.tobytes()
        for cut in (len(b), len(b) - 1, len(b) // 3):
            st, w = ref.unpacked_size(b[:cut])
            sz_in.append(np.frombuffer(b[:cut], np.uint8))
            sz_status.append(st)
            sz_words.append(w)

    def ragged(arrs, dtype):
        off = np.zeros(len(arrs) + 1, np.int64)
        off[1:] = np.cumsum([len(a) for a in arrs])
        data = np.concatenate([np.asarray(a, dtype) for a in arrs]) if arrs else np.zeros(0, dtype)
        return data, off

    out = {}
    for name, arrs, dt in (("chunk_in", chunk_in, "<u8"), ("chunk_out", chunk_out, np.uint8),
                           ("msg_in", msg_in, "<u8"), ("msg_out", msg_out, np.uint8),
                           ("rd_in", rd_in, np.uint8), ("rd_words", rd_words, "<u8"),
                           ("sz_in", sz_in, np.uint8)):
        out[name], out[name + "_off"] = ragged(arrs, dt)
    out["rd_status"] = np.array(rd_status, np.int32)
    out["rd_consumed"] = np.array(rd_consumed, np.int64)
    out["rd_limit"] = np.array(rd_limit, np.int64)
    out["sz_status"] = np.array(sz_status, np.int32)
    out["sz_words"] = np.array(sz_words, np.int64)
    dst = os.path.join(ROOT, "tests", "golden", "ref_vectors.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, os.path.getsize(dst), "bytes;",
          len(chunk_in), "chunks,", len(msg_in), "messages,", len(rd_in), "reads")


if __name__ == "__main__":
    main()
