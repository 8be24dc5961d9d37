#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of unpack index_kernel (run with CPK_STAMPS=1)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capnproto_amd  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
n, nseg, sw, prof = {"c2": (4096, 1, 8191, "flat"), "c3": (1 << 18, 1, 511, "flat"),
                     "c4": (32, 16, 524288, "pointer")}[cfg]
codec = capnproto_amd.Codec(0)
L = codec.lib
L.cpk_debug_stamps.argtypes = [C.c_int, C.POINTER(C.c_uint64)]
off, total = codec.gen_offsets(n, nseg=nseg, seg_words=sw, seed=20261015)
words = codec.gen_messages(prof, off, total, nseg=nseg, seed=20261015)
packed, moff, st = codec.pack_messages(words, off)
codec.sync()
P = int(moff[-1].item())
for rep in range(3):
    out = (C.c_uint64 * 16)()
    L.cpk_debug_stamps(2, out)
    codec.unpack_messages(packed, moff, total, nbytes=P)
    codec.sync()
    L.cpk_debug_stamps(2, out)
names = ["stage", "msg starts", "walk", "settle", "word counts+stores", "merge table", "tables"]
tiles = out[15] or 1
tot = sum(out[i] for i in range(7))
print(cfg, "tiles", tiles, "cycles/tile", round(tot / tiles))
for i, nm in enumerate(names):
    print(f"  {nm:20s} {out[i] / tiles:10.0f}  {100 * out[i] / max(tot, 1):5.1f}%")
