#!/usr/bin/env python3
"""Diagnostic: the stream split of a C5-shaped stream (1 Mi mixed messages), a few calls, for
rocprofv3 --kernel-trace --stats (per-kernel times of the split's phases)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capnproto_amd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
c = capnproto_amd.Codec(0)
off, total = c.gen_offsets(n, seed=7)
words = c.gen_messages("mixed", off, total, seed=7)
packed, poff, st = c.pack_messages(words, off)
c.sync()
nbytes = int(poff[-1].item())
import ctypes as C  # noqa: E402
L = capnproto_amd.load_library()
L.cpk_debug_split.restype = C.c_int
dbg = (C.c_uint64 * 8)()
for i in range(3):
    t0 = time.perf_counter()
    w2, woff, ioff, status, cnt = c.split_packed_stream(packed, total + 16, n + 1, nbytes=nbytes)
    c.sync()
    print("split ms", round(1e3 * (time.perf_counter() - t0), 2), "n", int(cnt.item()))
    assert L.cpk_debug_split(dbg) == 0
    print("  in-order pass: windows", dbg[0], "blocks", dbg[1], "serial guess/se/se2/walk/over",
          dbg[2], dbg[3], dbg[4], dbg[5], dbg[6])
