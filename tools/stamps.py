#!/usr/bin/env python3
"""Diagnostic: per-phase cycle breakdown of the tile kernels (run with CPK_STAMPS=1)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import capnproto_amd  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
sizes = {"c2": (4096, 1, 8191, "flat"), "c3": (1 << 18, 1, 511, "flat"),
         "c4": (32, 16, 524288, "pointer"), "c5": (200000, 1, 0, "mixed"),
         "c4b": (256, 16, 524288, "pointer")}[cfg]
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 20261015
codec = capnproto_amd.Codec(0)
L = codec.lib
L.cpk_debug_stamps.argtypes = [C.c_int, C.POINTER(C.c_uint64)]
n, nseg, sw, prof = sizes
off, total = codec.gen_offsets(n, nseg=nseg, seg_words=sw, seed=seed)
words = codec.gen_messages(prof, off, total, nseg=nseg, seed=seed)
packed, moff, st = codec.pack_messages(words, off)
codec.sync()
P = int(moff[-1].item())
codec.unpack_messages(packed, moff, total, nbytes=P)
codec.sync()
names = {0: ["passA", "lookahead+exit", "entry wait", "count+publish", "passB", "finish(prev)"],
         1: ["unsettled tiles", "table misses", "walk fails", "walks", "flagged msgs",
             "umask tiles", "merge steps (max/tile)", "settle iters", "walk records (sum)",
             "walk records (max/tile)", "merge walk > 64", "> 256", "> 1024", "settle > 8 rounds", "> 24"]}
for which in (0, 1):
    out = (C.c_uint64 * 16)()
    if L.cpk_debug_stamps(which, out) != 0:
        continue
    if which == 1:  # event counters of the unpack pipeline
        print("unpack counters:", {nm: out[i] for i, nm in enumerate(names[1])})
        nt = (P + 4095) // 4096
        print("per tile:", {nm: round(out[i] / nt, 2) for i, nm in enumerate(names[1]) if i >= 5})
        continue
    tiles = out[15] or 1
    tot = sum(out[i] for i in range(15))
    print(["pack", "unpack"][which], "tiles", out[15], "cycles/tile", tot / tiles)
    for i, nm in enumerate(names[which]):
        print(f"   {nm:22s} {out[i] / tiles:10.0f}  {100 * out[i] / max(tot, 1):5.1f}%")
